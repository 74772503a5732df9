#!/bin/bash
# Round 4, final build: the other workloads' bench lines (C2, C4, C5).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5z; mkdir -p $O
for wl in c2_final c4_bunny4k c5_mixed; do
  timeout -k 10 500 python bench.py --workload $wl --no-adaptive-leg > $O/bench_$wl.json 2> $O/bench_$wl.err || exit 1
  python3 scripts/sweep_summary.py $wl $O/bench_$wl.json
done
