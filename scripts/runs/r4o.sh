# round-3 end: the committed tree as the driver will run it (GPU tests, smoke, default bench line)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4o && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r4o/pytest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4o/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/r4o/bench_c3.json 2> gpurun_out/r4o/bench_c3.err
