# round-3 final: r4k (GPU tests, smoke, async-statistics A/B on C3 / C2), then the C2 profile and the C4 bench line
cd $GRAFT_REPO_ROOT && timeout -k 10 1000 bash scripts/r4k.sh && \
timeout -k 10 500 bash scripts/profile.sh r4l_c2 --schedule plain --workload c2_final && \
mkdir -p gpurun_out/r4l && timeout -k 10 300 python bench.py --workload c4_bunny4k > gpurun_out/r4l/bench_c4.json 2> gpurun_out/r4l/bench_c4.err
