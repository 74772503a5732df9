# round-3: the speculative walk adopted (PARK = 2 on trees of <= 65536 BVH4 nodes): GPU tests, then fixed-spp C3
# A/B (this build, the round-2 library, the round-2 speculative-walk variant) and the leaf-step schedule
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3g && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r3g/pytest.log 2>&1 && \
timeout -k 10 900 bash scripts/ab.sh r3g_c3 "--no-generic-leg" default 3360-ray-tracer_amd/variants/librtx_r2.so 3360-ray-tracer_amd/variants/librtx_spec8w.so && \
timeout -k 10 300 python bench.py --no-generic-leg --no-cpu-baseline --schedule park_step > gpurun_out/r3g/bench_c3_park_step.json 2> gpurun_out/r3g/bench_c3_park_step.err
