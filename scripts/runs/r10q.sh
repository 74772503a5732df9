#!/bin/bash
# Round 6 (r10q): the fixed-spp kernels' refill thresholds re-checked after the cheaper primary
# setup (FastDiv): PARK at 8 / 10 idle lanes (12 now) on C3, plain at 16 / 20 (24 now) on C2.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r10q; mkdir -p $O
V=3360-ray-tracer_amd/variants
timeout -k 10 600 bash scripts/ab.sh r10q_c3 "--no-generic-leg --no-adaptive-leg" default $V/librtx_rp8.so $V/librtx_rp10.so || exit 1
timeout -k 10 600 bash scripts/ab.sh r10q_c2 "--workload c2_final --no-generic-leg --no-adaptive-leg" default $V/librtx_rl16.so $V/librtx_rl20.so || exit 1
cp gpurun_out/ab_r10q_*.txt $O/
echo done
