# round-3 experiment: adaptive sub-renders offset (sub-render 1's phase 2 after sub-render 0's) vs lockstep vs one
# sub-render; C3 adaptive, interleaved rounds; then a kernel trace of each arm (timeline of the phases)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3t && OUT=gpurun_out/r3t/ab_offset_c3a.txt && : > $OUT && \
for round in 1 2; do
  for arm in "RTX_ADAPT_OFFSET=1" "RTX_ADAPT_OFFSET=0" "RTX_ADAPT_SUBS=1"; do
    res=$(env $arm timeout -k 10 300 python bench.py --no-cpu-baseline --no-generic-leg --adaptive --schedule park 2>>gpurun_out/r3t/ab.err) || exit $?
    echo "round $round $arm $(echo "$res" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.1f Mrays/s ms/step %.3f" % (d["value"], d["ms_per_step"]))')" >> $OUT
  done
done && cat $OUT && \
export TMPDIR=/tmp && \
for arm in 1 0; do
  RTX_ADAPT_OFFSET=$arm timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r3t/trace_off$arm -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-generic-leg --adaptive --schedule park --steps 3 --warmup 1 > gpurun_out/r3t/trace_off$arm.json 2> gpurun_out/r3t/trace_off$arm.err || exit $?
done
