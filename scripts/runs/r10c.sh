#!/bin/bash
# Round 6 (r10c): the block-shared chunk word decoded in 32-bit arithmetic (first slot | size |
# cursor): GPU suite, then A/B against the previous word (oldword) and chunk sizes 64 / 256 on C3
# adaptive, C2 adaptive and the fixed frame's samples through the phase kernel (min_spp = spp).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r10c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
V=3360-ray-tracer_amd/variants
L="$V/librtx_oldword.so default $V/librtx_cs64.so $V/librtx_cs256.so"
timeout -k 10 600 bash scripts/ab.sh r10c_c3a "--adaptive --no-generic-leg --no-adaptive-leg --steps 200" $L || exit 1
timeout -k 10 600 bash scripts/ab.sh r10c_c2a "--workload c2_final --adaptive --no-generic-leg --no-adaptive-leg --steps 150" $L || exit 1
timeout -k 10 600 bash scripts/ab.sh r10c_map1u "--adaptive --min-spp 200 --no-generic-leg --no-adaptive-leg --schedule park" "$V/librtx_oldword.so" default || exit 1
cp gpurun_out/ab_r10c_*.txt $O/
echo done
