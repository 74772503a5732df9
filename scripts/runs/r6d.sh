#!/bin/bash
# Round 4, final build: the 4-rank rehearsal of bench.py's N > 1 path on one GPU (32 spp).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
NPROC=4 timeout -k 10 450 bash scripts/multirank_rehearsal.sh --spp 32 || exit 1
mkdir -p gpurun_out/r6d && cp gpurun_out/bench_rehearsal_4rank.json gpurun_out/bench_rehearsal_4rank.err gpurun_out/r6d/
tail -1 gpurun_out/r6d/bench_rehearsal_4rank.json | cut -c1-200
