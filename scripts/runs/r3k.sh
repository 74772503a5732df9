# round-3 diagnostic: the batch queue's counters (variant build with RTX_AQ_STATS), adaptive C3; then the
# product's adaptive tests and C3 / C2 adaptive benches
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3k && \
RTX_DEBUG_ADAPT=1 RTX_LIB=$PWD/3360-ray-tracer_amd/variants/librtx_aqstats.so timeout -k 10 300 python bench.py --adaptive --no-generic-leg --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r3k/c3.json 2> gpurun_out/r3k/c3.err && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu -k "adaptive or parked or defocus" > gpurun_out/r3k/pytest_adaptive.log 2>&1 && \
timeout -k 10 300 python bench.py --adaptive --no-generic-leg --no-cpu-baseline > gpurun_out/r3k/c3_queue.json 2> gpurun_out/r3k/c3_queue.err && \
timeout -k 10 300 python bench.py --adaptive --no-generic-leg --no-cpu-baseline --workload c2_final > gpurun_out/r3k/c2_queue.json 2> gpurun_out/r3k/c2_queue.err
