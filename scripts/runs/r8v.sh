#!/bin/bash
# Round 5 (r8v): kernel trace of the C3 adaptive frame with the final policy (pooled prediction).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8v; mkdir -p $O
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$R/$O/trace" -o run --output-format csv -- python3 "$R/bench.py" --adaptive --no-cpu-baseline --no-generic-leg --schedule park > "$R/$O/trace_bench.json" 2> "$R/$O/trace.err" || exit 1
RTX_DEBUG_HOST=1 timeout -k 10 120 python3 "$R/bench.py" --adaptive --no-cpu-baseline --no-generic-leg --schedule park --steps 20 > "$R/$O/host.json" 2> "$R/$O/host.err" || exit 1
grep "rtx host" "$R/$O/host.err" | tail -5
