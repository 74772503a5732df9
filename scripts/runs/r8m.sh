#!/bin/bash
# Round 5 (r8m): the C4 adaptive band check's differing pixels (sample counts 11 segments apart in
# r8h / r8l): which pixels, and whether parity precision reproduces the oracle there.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8m; mkdir -p $O
timeout -k 10 600 python -u scripts/diag_adaptive_mismatch.py --workload c4_bunny4k --rows 529 1631 > $O/diag_c4.txt 2>&1 || { tail -20 $O/diag_c4.txt; exit 1; }
cat $O/diag_c4.txt
