cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3a && \
timeout -k 10 300 python bench.py --adaptive --no-generic-leg > gpurun_out/r3a/bench_c3_adaptive.json 2> gpurun_out/r3a/bench_c3_adaptive.err && \
timeout -k 10 300 python bench.py --adaptive --no-generic-leg --workload c2_final > gpurun_out/r3a/bench_c2_adaptive.json 2> gpurun_out/r3a/bench_c2_adaptive.err && \
export TMPDIR=/tmp && cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3a/prof_c3_adaptive -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --adaptive --no-cpu-baseline --no-generic-leg --steps 2 --warmup 1 --schedule park > $GRAFT_REPO_ROOT/gpurun_out/r3a/bench_c3_adaptive_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/r3a/prof.err
