#!/bin/bash
# Round 4: the uniform-group launches' chunk (256 default / 512 / 192 slots) on fixed C3 and C2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 800 bash scripts/ab.sh r6e_chunk0_c3 "--no-generic-leg --no-adaptive-leg" default \
  3360-ray-tracer_amd/variants/librtx_chunk0_512.so 3360-ray-tracer_amd/variants/librtx_chunk0_192.so > /dev/null || exit 1
cat gpurun_out/ab_r6e_chunk0_c3.txt
timeout -k 10 800 bash scripts/ab.sh r6e_chunk0_c2 "--workload c2_final --no-generic-leg --no-adaptive-leg" default \
  3360-ray-tracer_amd/variants/librtx_chunk0_512.so 3360-ray-tracer_amd/variants/librtx_chunk0_192.so > /dev/null || exit 1
cat gpurun_out/ab_r6e_chunk0_c2.txt
