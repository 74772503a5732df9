#!/bin/bash
# Round 4: A/B of two variant builds against the product on C3 (fixed, adaptive): the camera-only
# argument refill of the bunny's Lambertian texture-free builds (round 3's unmeasured r4n) and
# the quantised 64-byte BVH4 nodes (RTX_QNODE); the QNode build's parity on the fast-walk tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5b; mkdir -p $O
RTX_LIB=$PWD/3360-ray-tracer_amd/variants/librtx_qnode.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "fast_matches_parity or persistent_schedule_equals or parked_traversal" > $O/pytest_qnode.log 2>&1 || exit 1
timeout -k 10 600 bash scripts/ab.sh r5b_qnode_c3 "--no-generic-leg --no-adaptive-leg" default 3360-ray-tracer_amd/variants/librtx_qnode.so > /dev/null || exit 1
timeout -k 10 600 bash scripts/ab.sh r5b_camkarg_c3 "--no-generic-leg --no-adaptive-leg" default 3360-ray-tracer_amd/variants/librtx_camkarg.so > /dev/null || exit 1
timeout -k 10 600 bash scripts/ab.sh r5b_camkarg_c3a "--no-generic-leg --adaptive" default 3360-ray-tracer_amd/variants/librtx_camkarg.so > /dev/null || exit 1
echo done
