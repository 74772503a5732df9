# round-3: GPU tests (continue to the benches when tests merely fail: rc 1), then benches + adaptive profile
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3c && \
{ timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r3c/pytest.log 2>&1; rc=$?; [ $rc -le 1 ]; } && \
timeout -k 10 300 python bench.py --no-generic-leg > gpurun_out/r3c/bench_c3.json 2> gpurun_out/r3c/bench_c3.err && \
RTX_DEBUG_ADAPT=1 timeout -k 10 300 python bench.py --adaptive --no-generic-leg --steps 20 > gpurun_out/r3c/bench_c3_adaptive.json 2> gpurun_out/r3c/bench_c3_adaptive.err && \
timeout -k 10 300 python bench.py --adaptive --no-generic-leg --workload c2_final > gpurun_out/r3c/bench_c2_adaptive.json 2> gpurun_out/r3c/bench_c2_adaptive.err && \
export TMPDIR=/tmp && cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3c/prof_c3_adaptive -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --adaptive --no-cpu-baseline --no-generic-leg --steps 3 --warmup 1 --schedule park > $GRAFT_REPO_ROOT/gpurun_out/r3c/bench_c3_adaptive_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/r3c/prof.err
