#!/bin/bash
# Round 6 (r10x): wave priority around loads, split by site.  n1: node visit (priority 0 while
# the node's loads issue, 1 after); l1 / l2: leaf test (0 while the primitive loads issue,
# 1 / 2 after); n1l1, n1l2 both.  C3 and C2 fixed, C3 adaptive; interleaved.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
V=3360-ray-tracer_amd/variants
timeout -k 10 900 bash scripts/ab.sh prio_c3 "" default $V/librtx_n1.so $V/librtx_l1.so $V/librtx_n1l1.so $V/librtx_n1l2.so || exit 1
timeout -k 10 900 bash scripts/ab.sh prio_c2 "--workload c2_final" default $V/librtx_n1.so $V/librtx_l1.so $V/librtx_n1l1.so $V/librtx_n1l2.so || exit 1
timeout -k 10 900 bash scripts/ab.sh prio_c3a "--adaptive --no-generic-leg --no-adaptive-leg" default $V/librtx_n1.so $V/librtx_n1l1.so || exit 1
echo done
