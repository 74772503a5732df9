# round-3 experiment: adaptive on one launch (variant from branch wip-adaptive-queue): counters incl. lane occupancy
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3r && \
RTX_DEBUG_ADAPT=1 RTX_LIB=$PWD/3360-ray-tracer_amd/variants/librtx_q2stats.so timeout -k 10 300 python bench.py --adaptive --no-generic-leg --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r3r/c3_stats.json 2> gpurun_out/r3r/c3_stats.err
