#!/bin/bash
# Round 6 (r10i): does the counting builds' region timing perturb the product kernels (their ISA
# differs by register allocation)?  A/B of the build before it (46797c8) against the current one
# on C3 fixed and adaptive, and C2 fixed.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r10i; mkdir -p $O
V=3360-ray-tracer_amd/variants
timeout -k 10 600 bash scripts/ab.sh r10i_c3 "--no-generic-leg --no-adaptive-leg" $V/librtx_c46797c.so default || exit 1
timeout -k 10 600 bash scripts/ab.sh r10i_c3a "--adaptive --no-generic-leg --no-adaptive-leg --steps 200" $V/librtx_c46797c.so default || exit 1
timeout -k 10 600 bash scripts/ab.sh r10i_c2 "--workload c2_final --no-generic-leg --no-adaptive-leg" $V/librtx_c46797c.so default || exit 1
cp gpurun_out/ab_r10i_*.txt $O/
echo done
