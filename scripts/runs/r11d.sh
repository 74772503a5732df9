#!/bin/bash
# Round 6 (r11d): the product with the load barriers (node and primitive loads) and the walk /
# shading wave priorities: GPU suite, smoke, then A/B against the previous product (prev) on
# C2, C4, C5 fixed and C2, C4, C5 adaptive, interleaved.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
V=3360-ray-tracer_amd/variants
O=gpurun_out/r11d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
N="--no-generic-leg --no-adaptive-leg"
for w in c2_final c4_bunny4k c5_mixed; do
  timeout -k 10 900 bash scripts/ab.sh r11d_$w "--workload $w $N" $V/librtx_prev.so default || exit 1
  timeout -k 10 900 bash scripts/ab.sh r11d_${w}_a "--workload $w --adaptive $N" $V/librtx_prev.so default || exit 1
done
echo done
