# round-3: fixed-spp C3 A/B (this build, the round-2 library, the speculative-walk variant), adaptive C3/C2 +
# trace, then the GPU tests once with the speculative-walk variant
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3d && \
timeout -k 10 900 bash scripts/ab.sh r3d_c3 "--no-generic-leg" default 3360-ray-tracer_amd/variants/librtx_r2.so 3360-ray-tracer_amd/variants/librtx_spec8w.so && \
RTX_DEBUG_ADAPT=1 timeout -k 10 300 python bench.py --adaptive --no-generic-leg > gpurun_out/r3d/bench_c3_adaptive.json 2> gpurun_out/r3d/bench_c3_adaptive.err && \
timeout -k 10 300 python bench.py --adaptive --no-generic-leg --workload c2_final > gpurun_out/r3d/bench_c2_adaptive.json 2> gpurun_out/r3d/bench_c2_adaptive.err && \
export TMPDIR=/tmp && cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3d/prof_c3_adaptive -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --adaptive --no-cpu-baseline --no-generic-leg --steps 3 --warmup 1 --schedule park > $GRAFT_REPO_ROOT/gpurun_out/r3d/bench_c3_adaptive_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/r3d/prof.err && \
cd $GRAFT_REPO_ROOT && { RTX_LIB=$PWD/3360-ray-tracer_amd/variants/librtx_spec8w.so timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r3d/pytest_spec8w.log 2>&1; rc=$?; [ $rc -le 1 ]; }
