#!/bin/bash
# Round 4: block-shared chunk size, smaller: 128 (default now) / 64 / 32 slots.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 1000 bash scripts/ab.sh r5t_chunk_c3a "--adaptive --no-generic-leg" default \
  3360-ray-tracer_amd/variants/librtx_chunk64.so 3360-ray-tracer_amd/variants/librtx_chunk32.so > /dev/null || exit 1
cat gpurun_out/ab_r5t_chunk_c3a.txt
