#!/bin/bash
# Round 6 (r11e): ovl: the speculative walk issues a node's loads before the iteration's leaf
# test and finishes the visit after it, so the node's latency overlaps the primitive test
# (128 VGPRs, 11 spilled dwords outside the walk).  C3 fixed, C3 adaptive, C4, interleaved.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
V=3360-ray-tracer_amd/variants
N="--no-generic-leg --no-adaptive-leg"
timeout -k 10 900 bash scripts/ab.sh r11e_c3 "$N" default $V/librtx_ovl.so || exit 1
timeout -k 10 900 bash scripts/ab.sh r11e_c3a "--adaptive $N" default $V/librtx_ovl.so || exit 1
timeout -k 10 900 bash scripts/ab.sh r11e_c4 "--workload c4_bunny4k $N" default $V/librtx_ovl.so || exit 1
echo done
