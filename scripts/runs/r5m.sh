#!/bin/bash
# Round 4: rocprofv3 kernel-trace + PMC passes with the scene's schedule forced (so the trace
# holds only frame launches): C3 fixed and adaptive, the quantised-node variant, C2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 700 bash scripts/profile.sh r5m_c3 --schedule park || exit 1
echo "c3 profiled"
timeout -k 10 700 bash scripts/profile.sh r5m_c3a --schedule park --adaptive || exit 1
echo "c3a profiled"
RTX_LIB=$PWD/3360-ray-tracer_amd/variants/librtx_qnode.so timeout -k 10 700 bash scripts/profile.sh r5m_c3_qnode --schedule park || exit 1
echo "qnode profiled"
timeout -k 10 700 bash scripts/profile.sh r5m_c2 --schedule plain --workload c2_final || exit 1
echo done
