# round-3: record kernel (product-form convergence pre-check, 8 samples in flight) vs the pre-change
# library on C3 / C2 adaptive (one sub-render, phase floor 2^23 in both), C2 fixed spp (plain build ISA
# differs by one block order), then the adaptive GPU tests
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3z && \
RTX_ADAPT_SUBS=1 RTX_ADAPT_PHASE_SLOTS_LOG2=23 timeout -k 10 600 bash scripts/ab.sh r3z_c3a "--no-generic-leg --adaptive --schedule park" default 3360-ray-tracer_amd/variants/librtx_base.so && \
RTX_ADAPT_SUBS=1 RTX_ADAPT_PHASE_SLOTS_LOG2=23 timeout -k 10 600 bash scripts/ab.sh r3z_c2a "--no-generic-leg --adaptive --workload c2_final" default 3360-ray-tracer_amd/variants/librtx_base.so && \
timeout -k 10 600 bash scripts/ab.sh r3z_c2 "--no-generic-leg --workload c2_final" default 3360-ray-tracer_amd/variants/librtx_base.so && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_timed.py -m gpu -k "adaptive or recorded" > gpurun_out/r3z/pytest.log 2>&1
