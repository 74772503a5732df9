# round-3 check of the adaptive phase scheduler: targeted GPU tests, then C3/C2 adaptive benches
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3b && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "adaptive_phases" > gpurun_out/r3b/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --adaptive --no-generic-leg > gpurun_out/r3b/bench_c3_adaptive.json 2> gpurun_out/r3b/bench_c3_adaptive.err && \
timeout -k 10 300 python bench.py --adaptive --no-generic-leg --workload c2_final > gpurun_out/r3b/bench_c2_adaptive.json 2> gpurun_out/r3b/bench_c2_adaptive.err && \
timeout -k 10 300 python bench.py --no-generic-leg --no-cpu-baseline > gpurun_out/r3b/bench_c3.json 2> gpurun_out/r3b/bench_c3.err && \
export TMPDIR=/tmp && cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3b/prof_c3_adaptive -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --adaptive --no-cpu-baseline --no-generic-leg --steps 3 --warmup 1 --schedule park > $GRAFT_REPO_ROOT/gpurun_out/r3b/bench_c3_adaptive_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/r3b/prof.err
