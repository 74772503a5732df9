# round-3: adaptive phases with the next-phase batch floor (k_adapt_floor), A/B against the previous build
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3n && \
RTX_DEBUG_ADAPT=1 RTX_ADAPT_SUBS=1 timeout -k 10 300 python bench.py --adaptive --no-generic-leg --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r3n/dbg_s1.json 2> gpurun_out/r3n/dbg_s1.err && \
timeout -k 10 600 bash scripts/ab.sh r3n_c3a "--no-generic-leg --adaptive" default 3360-ray-tracer_amd/variants/librtx_base.so && \
timeout -k 10 600 bash scripts/ab.sh r3n_c2a "--no-generic-leg --adaptive --workload c2_final" default 3360-ray-tracer_amd/variants/librtx_base.so && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu -k "adaptive" > gpurun_out/r3n/pytest_adaptive.log 2>&1
