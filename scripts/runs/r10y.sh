#!/bin/bash
# Round 6 (r10y): what the node-visit priority does.  n1: priority 0 while the node's loads
# issue, 1 after; n2: 2 while they issue, 0 after; n3: 0 and 0 (the instructions, no priority
# change); n1s0 / n1s2: n1, and priority 0 / 2 from the end of the walk (shading, refill) to
# the next node visit.  C3 all six; C4 and C5 default against n1.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
V=3360-ray-tracer_amd/variants
timeout -k 10 900 bash scripts/ab.sh prio3_c3 "--no-generic-leg --no-adaptive-leg" default $V/librtx_n1.so $V/librtx_n2.so $V/librtx_n3.so $V/librtx_n1s0.so $V/librtx_n1s2.so || exit 1
timeout -k 10 900 bash scripts/ab.sh prio3_c4 "--workload c4_bunny4k --no-generic-leg --no-adaptive-leg" default $V/librtx_n1.so || exit 1
timeout -k 10 900 bash scripts/ab.sh prio3_c5 "--workload c5_mixed --no-generic-leg --no-adaptive-leg" default $V/librtx_n1.so || exit 1
echo done
