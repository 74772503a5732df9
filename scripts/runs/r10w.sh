#!/bin/bash
# Round 6 (r10w): wave priority (s_setprio) around the node loads of a BVH4 visit.
# prio1: priority 2 while the node's loads issue, 0 after; prio2: 0 while they issue, 1 for the
# slab tests, sort and push.  C3 (PARK kernel) and C2 (plain kernel), fixed spp, interleaved.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
V=3360-ray-tracer_amd/variants
timeout -k 10 900 bash scripts/ab.sh prio_c3 "" default $V/librtx_prio1.so $V/librtx_prio2.so || exit 1
timeout -k 10 900 bash scripts/ab.sh prio_c2 "--workload c2_final" default $V/librtx_prio1.so $V/librtx_prio2.so || exit 1
echo done
