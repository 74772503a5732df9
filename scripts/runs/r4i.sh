# round-3 final build: GPU tests + smoke, the default and adaptive bench lines, then profiles (r4h)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4i && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r4i/pytest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4i/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/r4i/bench_c3.json 2> gpurun_out/r4i/bench_c3.err && \
timeout -k 10 600 python bench.py --adaptive > gpurun_out/r4i/bench_c3a.json 2> gpurun_out/r4i/bench_c3a.err && \
timeout -k 10 400 python bench.py --workload c2_final --no-cpu-baseline > gpurun_out/r4i/bench_c2.json 2> gpurun_out/r4i/bench_c2.err && \
timeout -k 10 700 bash scripts/profile.sh r4h_c3 --schedule park && \
timeout -k 10 700 bash scripts/profile.sh r4h_c3a --schedule park --adaptive
