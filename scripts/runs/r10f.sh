#!/bin/bash
# Round 6 (r10f): hybrid slot claims in the adaptive phase kernel (a private register chunk while
# the wave's region has more than T slots left, block-shared LDS chunks for the region's last T):
# A/B of T = 128k / 256k / 512k against the product on C3 and C2 adaptive and the fixed frame's
# samples through the phase kernel.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r10f; mkdir -p $O
V=3360-ray-tracer_amd/variants
L="default $V/librtx_hy128k.so $V/librtx_hy256k.so $V/librtx_hy512k.so"
timeout -k 10 600 bash scripts/ab.sh r10f_c3a "--adaptive --no-generic-leg --no-adaptive-leg --steps 200" $L || exit 1
timeout -k 10 600 bash scripts/ab.sh r10f_c2a "--workload c2_final --adaptive --no-generic-leg --no-adaptive-leg --steps 150" $L || exit 1
timeout -k 10 600 bash scripts/ab.sh r10f_map1u "--adaptive --min-spp 200 --no-generic-leg --no-adaptive-leg --schedule park" default $V/librtx_hy256k.so || exit 1
cp gpurun_out/ab_r10f_*.txt $O/
echo done
