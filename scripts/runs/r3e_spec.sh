# round-3: the speculative PARK walk (RTX_LEAF_SPEC=8, wait rule, leaf round at >= 8 lanes) as a variant
# library: the GPU tests once with it, then C3 A/B against the default build
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3e && \
{ RTX_LIB=$PWD/3360-ray-tracer_amd/variants/librtx_spec8w.so timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r3e/pytest_spec8w.log 2>&1; rc=$?; [ $rc -le 1 ]; } && \
timeout -k 10 900 bash scripts/ab.sh r3e_spec8w_c3 "--no-generic-leg" default 3360-ray-tracer_amd/variants/librtx_spec8w.so
