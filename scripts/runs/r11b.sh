#!/bin/bash
# Round 6 (r11b): shading without the dependent record load (m: kind from the build or the
# global primitives' kinds, material from the walk), alone and with the load barriers + phase
# priorities (bwslm).  GPU suite on bwslm first (parity), then C3 fixed A/B, interleaved.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
V=3360-ray-tracer_amd/variants
O=gpurun_out/r11b; mkdir -p $O
RTX_LIB=$R/$V/librtx_bwslm.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_bwslm.log 2>&1 || { tail -30 $O/pytest_gpu_bwslm.log; exit 1; }
tail -1 $O/pytest_gpu_bwslm.log
timeout -k 10 900 bash scripts/ab.sh r11b_c3 "--no-generic-leg --no-adaptive-leg" default $V/librtx_m.so $V/librtx_bwslm.so || exit 1
echo done
