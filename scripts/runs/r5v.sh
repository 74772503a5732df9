#!/bin/bash
# Round 4: one init launch per frame / per adaptive launch instead of fills: parity, then A/B
# against the previous build (variants/librtx_prev.so), adaptive and fixed C3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5v; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_timed.py \
  -k "adaptive or banded or render_multi or group_size" > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 bash scripts/ab.sh r5v_init_c3a "--adaptive --no-generic-leg" default 3360-ray-tracer_amd/variants/librtx_prev.so > /dev/null || exit 1
cat gpurun_out/ab_r5v_init_c3a.txt
timeout -k 10 600 bash scripts/ab.sh r5v_init_c3 "--no-generic-leg --no-adaptive-leg" default 3360-ray-tracer_amd/variants/librtx_prev.so > /dev/null || exit 1
cat gpurun_out/ab_r5v_init_c3.txt
