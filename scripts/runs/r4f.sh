# round-3: the primary's inputs read from the kernel argument segment at refill (SGPR spills 79 -> 60 on C3,
# scratch 52 -> 0 B; C5 80 -> 16 B): GPU tests, then A/B against the HEAD library on C3, C2, C5 (256 spp),
# the C3 generic build and C3 adaptive
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4f && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r4f/pytest.log 2>&1 && \
timeout -k 10 600 bash scripts/ab.sh r4f_c3 "--no-generic-leg" default 3360-ray-tracer_amd/variants/librtx_base.so && \
timeout -k 10 600 bash scripts/ab.sh r4f_c2 "--no-generic-leg --workload c2_final" default 3360-ray-tracer_amd/variants/librtx_base.so && \
timeout -k 10 600 bash scripts/ab.sh r4f_c5 "--no-generic-leg --workload c5_mixed --spp 256" default 3360-ray-tracer_amd/variants/librtx_base.so && \
timeout -k 10 600 bash scripts/ab.sh r4f_c3gen "--no-generic-leg --generic" default 3360-ray-tracer_amd/variants/librtx_base.so && \
timeout -k 10 600 bash scripts/ab.sh r4f_c3a "--no-generic-leg --adaptive" default 3360-ray-tracer_amd/variants/librtx_base.so
