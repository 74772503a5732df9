# round-3: lockstep sub-renders (offset removed), recorded-segment counting (ABI 6): the adaptive GPU tests,
# the adaptive bench line (value on recorded segments), then a phase-floor / sub-render A/B (frame time)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3x && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_timed.py -m gpu -k "adaptive or recorded" > gpurun_out/r3x/pytest.log 2>&1 && \
timeout -k 10 600 python bench.py --adaptive > gpurun_out/r3x/bench_c3a.json 2> gpurun_out/r3x/bench_c3a.err && \
OUT=gpurun_out/r3x/ab_adapt_floor2_c3a.txt && : > $OUT && \
for round in 1 2; do
  for arm in "RTX_ADAPT_PHASE_SLOTS_LOG2=21" "RTX_ADAPT_PHASE_SLOTS_LOG2=22" "RTX_ADAPT_PHASE_SLOTS_LOG2=23" "RTX_ADAPT_PHASE_SLOTS_LOG2=24" "RTX_ADAPT_SUBS=1 RTX_ADAPT_PHASE_SLOTS_LOG2=21" "RTX_ADAPT_SUBS=1 RTX_ADAPT_PHASE_SLOTS_LOG2=23"; do
    res=$(env $arm timeout -k 10 300 python bench.py --no-cpu-baseline --no-generic-leg --adaptive --schedule park 2>>gpurun_out/r3x/ab.err) || exit $?
    echo "round $round $arm $(echo "$res" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.1f Mrays/s (traced %.1f) ms/step %.3f" % (d["value"], d["traced_value"], d["ms_per_step"]))')" >> $OUT
  done
done && cat $OUT && \
OUT=gpurun_out/r3x/ab_adapt_floor2_c2a.txt && : > $OUT && \
for arm in "RTX_ADAPT_PHASE_SLOTS_LOG2=21" "RTX_ADAPT_PHASE_SLOTS_LOG2=23"; do
  res=$(env $arm timeout -k 10 300 python bench.py --no-cpu-baseline --no-generic-leg --adaptive --workload c2_final 2>>gpurun_out/r3x/ab.err) || exit $?
  echo "$arm $(echo "$res" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.1f Mrays/s (traced %.1f) ms/step %.3f" % (d["value"], d["traced_value"], d["ms_per_step"]))')" >> $OUT
done && cat $OUT
