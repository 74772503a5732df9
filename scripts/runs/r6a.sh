#!/bin/bash
# Round 4: the adaptive record's loads in flight per lane (8 default / 16 / 32), with a kernel
# trace of each arm's record times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 1000 bash scripts/ab.sh r6a_recahead_c3a "--adaptive --no-generic-leg" default \
  3360-ray-tracer_amd/variants/librtx_rec16.so 3360-ray-tracer_amd/variants/librtx_rec32.so > /dev/null || exit 1
cat gpurun_out/ab_r6a_recahead_c3a.txt
