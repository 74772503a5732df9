# round-3: the primary's inputs read from the kernel argument segment at refill (SGPR spills 79 -> 60 on C3,
# scratch 52 -> 0 B; C5 80 -> 16 B): GPU tests + smoke, A/B against the HEAD library (C3, C2, C5 at
# 256 spp, the C3 generic build, C3 adaptive), then the default and adaptive bench lines
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4g && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r4g/pytest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4g/smoke.log 2>&1 && \
timeout -k 10 600 bash scripts/ab.sh r4g_c3 "--no-generic-leg" default 3360-ray-tracer_amd/variants/librtx_base.so && \
timeout -k 10 600 bash scripts/ab.sh r4g_c2 "--no-generic-leg --workload c2_final" default 3360-ray-tracer_amd/variants/librtx_base.so && \
timeout -k 10 600 bash scripts/ab.sh r4g_c5 "--no-generic-leg --workload c5_mixed --spp 256 --steps 3 --warmup 1" default 3360-ray-tracer_amd/variants/librtx_base.so && \
timeout -k 10 600 bash scripts/ab.sh r4g_c3gen "--no-generic-leg --generic" default 3360-ray-tracer_amd/variants/librtx_base.so && \
timeout -k 10 600 bash scripts/ab.sh r4g_c3a "--no-generic-leg --adaptive" default 3360-ray-tracer_amd/variants/librtx_base.so && \
timeout -k 10 600 python bench.py > gpurun_out/r4g/bench_c3.json 2> gpurun_out/r4g/bench_c3.err && \
timeout -k 10 600 python bench.py --adaptive > gpurun_out/r4g/bench_c3a.json 2> gpurun_out/r4g/bench_c3a.err
