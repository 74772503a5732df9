#!/bin/bash
# Round 4, final build: the C4 line (PARK kernels with 512-slot chunks).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6f; mkdir -p $O
timeout -k 10 500 python bench.py --workload c4_bunny4k --no-adaptive-leg > $O/bench_c4_bunny4k.json 2> $O/bench_c4_bunny4k.err || exit 1
python3 scripts/sweep_summary.py c4 $O/bench_c4_bunny4k.json
