#!/bin/bash
# Round 4: the block-shared chunk size of the adaptive phase launches (128 / 256 / 512 slots).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 1000 bash scripts/ab.sh r5r_chunk_c3a "--adaptive --no-generic-leg" default \
  3360-ray-tracer_amd/variants/librtx_chunk128.so 3360-ray-tracer_amd/variants/librtx_chunk512.so > /dev/null || exit 1
cat gpurun_out/ab_r5r_chunk_c3a.txt
