# round-3 re-entry check of HEAD (offset adaptive sub-renders): GPU tests, smoke, the default bench line,
# C3 adaptive with offset vs lockstep sub-renders
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3u && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r3u/pytest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3u/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/r3u/bench_c3.json 2> gpurun_out/r3u/bench_c3.err && \
timeout -k 10 600 python bench.py --adaptive > gpurun_out/r3u/bench_c3a.json 2> gpurun_out/r3u/bench_c3a.err && \
RTX_ADAPT_OFFSET=0 timeout -k 10 300 python bench.py --adaptive --no-cpu-baseline --no-generic-leg > gpurun_out/r3u/bench_c3a_off0.json 2> gpurun_out/r3u/bench_c3a_off0.err && \
RTX_ADAPT_OFFSET=1 timeout -k 10 300 python bench.py --adaptive --no-cpu-baseline --no-generic-leg > gpurun_out/r3u/bench_c3a_off1.json 2> gpurun_out/r3u/bench_c3a_off1.err
