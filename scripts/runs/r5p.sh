#!/bin/bash
# Round 4: launch timelines (counting build): slots used up vs waves end, fixed and adaptive.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5p; mkdir -p $O
RTX_DEBUG_DRAIN=1 RTX_DEBUG_ADAPT=1 timeout -k 10 300 python3 scripts/drain_timeline.py > $O/out.txt 2> $O/timeline.txt || { tail $O/timeline.txt; exit 1; }
grep -E "==|timeline|phase" $O/timeline.txt
