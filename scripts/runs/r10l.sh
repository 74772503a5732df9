#!/bin/bash
# Round 6 (r10l): launch-constant divisions (FastDiv: slot -> pixel by K, pixel -> row by the row
# length and the stripe height, one multiply-high each) in the working build: GPU suite, then A/B
# against the committed build (head) on C3 / C3 adaptive / C2 / C5 (256 spp); and the generic
# PARK builds with the restated small-argument cos/sin (in the working build too) on the generic C3
# frame.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r10l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
V=3360-ray-tracer_amd/variants
timeout -k 10 600 bash scripts/ab.sh r10l_c3 "--no-generic-leg --no-adaptive-leg" $V/librtx_head.so default || exit 1
timeout -k 10 600 bash scripts/ab.sh r10l_c3a "--adaptive --no-generic-leg --no-adaptive-leg --steps 200" $V/librtx_head.so default || exit 1
timeout -k 10 600 bash scripts/ab.sh r10l_c2 "--workload c2_final --no-generic-leg --no-adaptive-leg" $V/librtx_head.so default || exit 1
timeout -k 10 600 bash scripts/ab.sh r10l_c5 "--workload c5_mixed --no-generic-leg --no-adaptive-leg --spp 256" $V/librtx_head.so default || exit 1
timeout -k 10 600 bash scripts/ab.sh r10l_generic "--generic --no-generic-leg --no-adaptive-leg" $V/librtx_head.so default || exit 1
cp gpurun_out/ab_r10l_*.txt $O/
echo done
