#!/bin/bash
# Round 6 (r10j): the adaptive phase kernel's own speculative-walk thresholds (MAP 1 only): leaf
# rounds at 6 / 12 lanes holding leaves (8 now), parking at 12 / 20 walking lanes (16 now), on C3
# adaptive; the fixed-spp kernels are unchanged (ISA-identical).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r10j; mkdir -p $O
V=3360-ray-tracer_amd/variants
L="default $V/librtx_lm6.so $V/librtx_lm12.so $V/librtx_pk12.so $V/librtx_pk20.so"
timeout -k 10 900 bash scripts/ab.sh r10j_c3a "--adaptive --no-generic-leg --no-adaptive-leg --steps 200" $L || exit 1
cp gpurun_out/ab_r10j_*.txt $O/
echo done
