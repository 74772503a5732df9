#!/bin/bash
# Round 6 (r11h): rocprofv3 passes of the final build (load barriers, phase priority) for C4 and C5 (the bench's roofline for
# those workloads), and the 2-rank rehearsal of the N > 1 bench path on one GPU (C4, 32 spp).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r11h; mkdir -p $O
timeout -k 10 900 bash scripts/profile.sh r11h_c4 --workload c4_bunny4k --schedule park || exit 1
timeout -k 10 900 bash scripts/profile.sh r11h_c5 --workload c5_mixed --schedule plain || exit 1
NPROC=2 timeout -k 10 500 bash scripts/multirank_rehearsal.sh --spp 32 || { tail -20 gpurun_out/bench_rehearsal_2rank.err; exit 1; }
cp gpurun_out/bench_rehearsal_2rank.json $O/
tail -1 $O/bench_rehearsal_2rank.json | cut -c1-400
echo done
