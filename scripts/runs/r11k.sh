#!/bin/bash
# Round 6 (r11k): rf1: the refill (slot claim, primary ray) at the walk's priority 1 instead of
# shading's 0.  C3 fixed, C3 adaptive, C2, interleaved.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
V=3360-ray-tracer_amd/variants
N="--no-generic-leg --no-adaptive-leg"
timeout -k 10 900 bash scripts/ab.sh r11k_c3 "$N" default $V/librtx_rf1.so || exit 1
timeout -k 10 900 bash scripts/ab.sh r11k_c3a "--adaptive $N" default $V/librtx_rf1.so || exit 1
timeout -k 10 900 bash scripts/ab.sh r11k_c2 "--workload c2_final $N" default $V/librtx_rf1.so || exit 1
echo done
