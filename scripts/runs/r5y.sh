#!/bin/bash
# Round 4: the refill threshold of the adaptive (block-shared chunk) launches: 16 (the PARK
# kernel's, default) / 8 / 32 idle lanes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 1000 bash scripts/ab.sh r5y_refill_c3a "--adaptive --no-generic-leg" default \
  3360-ray-tracer_amd/variants/librtx_refill8.so 3360-ray-tracer_amd/variants/librtx_refill32.so > /dev/null || exit 1
cat gpurun_out/ab_r5y_refill_c3a.txt
