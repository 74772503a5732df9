# round-3: adaptive sampling on one persistent launch (batch queue): GPU tests, then adaptive C3 / C2 with the
# queue and with the phased scheduler (RTX_ADAPT_PHASES=1)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3j && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu -k "adaptive or parked or defocus" > gpurun_out/r3j/pytest_adaptive.log 2>&1 && \
timeout -k 10 300 python bench.py --adaptive --no-generic-leg --no-cpu-baseline > gpurun_out/r3j/c3_queue.json 2> gpurun_out/r3j/c3_queue.err && \
RTX_ADAPT_PHASES=1 timeout -k 10 300 python bench.py --adaptive --no-generic-leg --no-cpu-baseline > gpurun_out/r3j/c3_phases.json 2> gpurun_out/r3j/c3_phases.err && \
timeout -k 10 300 python bench.py --adaptive --no-generic-leg --no-cpu-baseline --workload c2_final > gpurun_out/r3j/c2_queue.json 2> gpurun_out/r3j/c2_queue.err && \
RTX_ADAPT_PHASES=1 timeout -k 10 300 python bench.py --adaptive --no-generic-leg --no-cpu-baseline --workload c2_final > gpurun_out/r3j/c2_phases.json 2> gpurun_out/r3j/c2_phases.err && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r3j/pytest_all.log 2>&1 && \
timeout -k 10 900 python scripts/calibrate_cpu.py --threads 16 --out gpurun_out/r3j/cpu_calibration_16t.json --host "GPU box host (MI355X pool), 16 threads" > gpurun_out/r3j/calibrate.out 2>&1
