#!/bin/bash
# Round 6 (r10z): the node loads issued together (a scheduling barrier after them, b) against
# the s_setprio forms, and wave priority by phase: walk 1, shading and refill 0 (ws).
# b: barrier only; bws: barrier + walk 1 / shade 0; bwsl: bws + a barrier after the primitive
# loads of a leaf test; n1s0: priority 0 during the node loads, 1 after, shading 0;
# n1ws: n1s0 with priority 1 set at the walk's start.  C3 fixed, interleaved.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
V=3360-ray-tracer_amd/variants
timeout -k 10 900 bash scripts/ab.sh prio4_c3 "--no-generic-leg --no-adaptive-leg" default $V/librtx_b.so $V/librtx_bws.so $V/librtx_bwsl.so $V/librtx_n1s0.so $V/librtx_n1ws.so || exit 1
echo done
