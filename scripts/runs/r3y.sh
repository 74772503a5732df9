# round-3: deferred texture lookups (textured builds: the lookup at the top of the next round): GPU tests,
# C5 (256 spp) and the C3 generic build against the pre-change library; adaptive: one sub-render and
# phase floors 2^23..2^25 / margin on C3, one vs two sub-renders on C2
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3y && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r3y/pytest.log 2>&1 && \
timeout -k 10 600 bash scripts/ab.sh r3y_c5 "--no-generic-leg --workload c5_mixed --spp 256" default 3360-ray-tracer_amd/variants/librtx_base.so && \
timeout -k 10 600 bash scripts/ab.sh r3y_c3gen "--no-generic-leg --generic" default 3360-ray-tracer_amd/variants/librtx_base.so && \
OUT=gpurun_out/r3y/ab_adapt_s1_c3a.txt && : > $OUT && \
for round in 1 2; do
  for arm in "RTX_ADAPT_SUBS=1 RTX_ADAPT_PHASE_SLOTS_LOG2=23" "RTX_ADAPT_SUBS=1 RTX_ADAPT_PHASE_SLOTS_LOG2=24" "RTX_ADAPT_SUBS=1 RTX_ADAPT_PHASE_SLOTS_LOG2=25" "RTX_ADAPT_SUBS=1 RTX_ADAPT_PHASE_SLOTS_LOG2=23 RTX_ADAPT_MARGIN_STEP=0.5" "RTX_ADAPT_SUBS=1 RTX_ADAPT_PHASE_SLOTS_LOG2=24 RTX_ADAPT_MARGIN_STEP=0.5"; do
    res=$(env $arm timeout -k 10 300 python bench.py --no-cpu-baseline --no-generic-leg --adaptive --schedule park 2>>gpurun_out/r3y/ab.err) || exit $?
    echo "round $round $arm $(echo "$res" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.1f Mrays/s (traced %.1f) ms/step %.3f" % (d["value"], d["traced_value"], d["ms_per_step"]))')" >> $OUT
  done
done && cat $OUT && \
OUT=gpurun_out/r3y/ab_adapt_s1_c2a.txt && : > $OUT && \
for arm in "RTX_ADAPT_SUBS=2 RTX_ADAPT_PHASE_SLOTS_LOG2=23" "RTX_ADAPT_SUBS=1 RTX_ADAPT_PHASE_SLOTS_LOG2=23" "RTX_ADAPT_SUBS=1 RTX_ADAPT_PHASE_SLOTS_LOG2=24"; do
  res=$(env $arm timeout -k 10 300 python bench.py --no-cpu-baseline --no-generic-leg --adaptive --workload c2_final 2>>gpurun_out/r3y/ab.err) || exit $?
  echo "$arm $(echo "$res" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.1f Mrays/s (traced %.1f) ms/step %.3f" % (d["value"], d["traced_value"], d["ms_per_step"]))')" >> $OUT
done && cat $OUT
