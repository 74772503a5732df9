#!/bin/bash
# Round 6 (r10m): FastDiv in the adaptive phase kernel (MAP 1) or only in the fixed-spp one:
# A/B of the committed build (head), the working build (FastDiv everywhere) and FastDiv only for
# MAP 0 (fd0map1) on C3 and C2 adaptive.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r10m; mkdir -p $O
V=3360-ray-tracer_amd/variants
L="$V/librtx_head.so default $V/librtx_fd0map1.so"
timeout -k 10 600 bash scripts/ab.sh r10m_c3a "--adaptive --no-generic-leg --no-adaptive-leg --steps 200" $L || exit 1
timeout -k 10 600 bash scripts/ab.sh r10m_c2a "--workload c2_final --adaptive --no-generic-leg --no-adaptive-leg --steps 150" $L || exit 1
cp gpurun_out/ab_r10m_*.txt $O/
echo done
