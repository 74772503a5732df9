# round-3: one adaptive sequence (sub-renders removed), phase floor 2^23, record kernel pre-check (8 in
# flight): GPU tests; adaptive C3 / C2 against the pre-change library (run with one sub-render and the
# same floor); the default bench line and the adaptive line
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4a && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r4a/pytest.log 2>&1 && \
RTX_ADAPT_SUBS=1 RTX_ADAPT_PHASE_SLOTS_LOG2=23 timeout -k 10 600 bash scripts/ab.sh r4a_c3a "--no-generic-leg --adaptive --schedule park" default 3360-ray-tracer_amd/variants/librtx_base.so && \
RTX_ADAPT_SUBS=1 RTX_ADAPT_PHASE_SLOTS_LOG2=23 timeout -k 10 600 bash scripts/ab.sh r4a_c2a "--no-generic-leg --adaptive --workload c2_final" default 3360-ray-tracer_amd/variants/librtx_base.so && \
timeout -k 10 600 python bench.py > gpurun_out/r4a/bench_c3.json 2> gpurun_out/r4a/bench_c3.err && \
timeout -k 10 600 python bench.py --adaptive > gpurun_out/r4a/bench_c3a.json 2> gpurun_out/r4a/bench_c3a.err && \
RTX_DEBUG_ADAPT=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-generic-leg --adaptive --steps 3 --warmup 1 > gpurun_out/r4a/debug_adapt.json 2> gpurun_out/r4a/debug_adapt.err
