# round-3: adaptive phases' pixels ordered largest batch first within each slot counter region
# (RTX_ADAPT_ORDER=0: pixel order) on C3 / C2 adaptive, interleaved rounds; then the adaptive GPU tests
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4c && \
for w in c3_bunny c2_final; do
  OUT=gpurun_out/r4c/ab_order_$w.txt && : > $OUT
  for round in 1 2 3; do
    for arm in 1 0; do
      res=$(RTX_ADAPT_ORDER=$arm timeout -k 10 300 python bench.py --no-cpu-baseline --no-generic-leg --adaptive --workload $w 2>>gpurun_out/r4c/ab.err) || exit $?
      echo "round $round RTX_ADAPT_ORDER=$arm $(echo "$res" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.1f Mrays/s (traced %.1f) ms/step %.3f" % (d["value"], d["traced_value"], d["ms_per_step"]))')" >> $OUT
    done
  done
done && cat gpurun_out/r4c/ab_order_*.txt && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_timed.py tests/test_gpu_parity.py -m gpu -k "adaptive or recorded" > gpurun_out/r4c/pytest.log 2>&1 && \
RTX_DEBUG_ADAPT=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-generic-leg --adaptive --steps 3 --warmup 1 > gpurun_out/r4c/debug_adapt.json 2> gpurun_out/r4c/debug_adapt.err
