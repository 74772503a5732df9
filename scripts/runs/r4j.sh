# round-3 final build: profiles of C2 (plain) and C5 (textured, 256 spp), then full bench lines of C4 and C5
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4j && \
timeout -k 10 700 bash scripts/profile.sh r4j_c2 --schedule plain --workload c2_final && \
timeout -k 10 700 bash scripts/profile.sh r4j_c5 --schedule plain --workload c5_mixed && \
timeout -k 10 600 python bench.py --workload c4_bunny4k > gpurun_out/r4j/bench_c4.json 2> gpurun_out/r4j/bench_c4.err && \
timeout -k 10 600 python bench.py --workload c5_mixed > gpurun_out/r4j/bench_c5.json 2> gpurun_out/r4j/bench_c5.err
