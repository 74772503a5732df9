# round-3: adaptive phase tuning A/B on C3 adaptive (PARK): smallest phase (log2 slots) and per-phase batch
# margin step, interleaved rounds; then a kernel trace of the default arm (phase timeline)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3v && OUT=gpurun_out/r3v/ab_adapt_tune_c3a.txt && : > $OUT && \
for round in 1 2; do
  for arm in "RTX_ADAPT_PHASE_SLOTS_LOG2=21" "RTX_ADAPT_PHASE_SLOTS_LOG2=22" "RTX_ADAPT_PHASE_SLOTS_LOG2=23" "RTX_ADAPT_MARGIN_STEP=0.5" "RTX_ADAPT_MARGIN_STEP=0.5 RTX_ADAPT_PHASE_SLOTS_LOG2=22" "RTX_ADAPT_MARGIN_STEP=0.1"; do
    res=$(env $arm timeout -k 10 300 python bench.py --no-cpu-baseline --no-generic-leg --adaptive --schedule park 2>>gpurun_out/r3v/ab.err) || exit $?
    echo "round $round $arm $(echo "$res" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.1f Mrays/s ms/step %.3f" % (d["value"], d["ms_per_step"]))')" >> $OUT
  done
done && cat $OUT && \
RTX_DEBUG_ADAPT=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-generic-leg --adaptive --schedule park --steps 3 --warmup 1 > gpurun_out/r3v/debug_adapt.json 2> gpurun_out/r3v/debug_adapt.err && \
export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r3v/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-generic-leg --adaptive --schedule park --steps 3 --warmup 1 > gpurun_out/r3v/trace.json 2> gpurun_out/r3v/trace.err
