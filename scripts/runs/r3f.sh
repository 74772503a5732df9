# round-3: per-phase rates of the adaptive scheduler (debug build path: syncs per phase), 1 vs 2 sub-renders;
# fixed-spp C3 at 16 spp (one launch the size of the adaptive first phase)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3f && \
RTX_DEBUG_ADAPT=1 RTX_ADAPT_SUBS=1 timeout -k 10 300 python bench.py --adaptive --no-generic-leg --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3f/dbg_s1.json 2> gpurun_out/r3f/dbg_s1.err && \
RTX_ADAPT_SUBS=1 timeout -k 10 300 python bench.py --adaptive --no-generic-leg --no-cpu-baseline > gpurun_out/r3f/bench_c3_adaptive_s1.json 2> gpurun_out/r3f/bench_c3_adaptive_s1.err && \
timeout -k 10 300 python bench.py --adaptive --no-generic-leg --no-cpu-baseline > gpurun_out/r3f/bench_c3_adaptive_s2.json 2> gpurun_out/r3f/bench_c3_adaptive_s2.err && \
timeout -k 10 300 python bench.py --spp 16 --no-generic-leg --no-cpu-baseline > gpurun_out/r3f/bench_c3_spp16.json 2> gpurun_out/r3f/bench_c3_spp16.err
