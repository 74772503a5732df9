#!/bin/bash
# Round 5 (r9c): the radiance records stored non-temporal (global_store ... nt, variant nt) so the
# 2.7 GB of records per C3 frame stream through the L2 instead of displacing the scene's nodes.
# Parity subset on nt, then C3 fixed / adaptive and C2 fixed, two interleaved rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r9c; mkdir -p $O
RTX_LIB=$R/3360-ray-tracer_amd/variants/librtx_nt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_parity.py -m gpu -x -q -k "bunny or c3 or schedule or final" --timeout 300 --timeout-method thread > $O/pytest_nt.log 2>&1 || { tail -30 $O/pytest_nt.log; exit 1; }
tail -1 $O/pytest_nt.log
for r in 1 2; do
  for v in product nt; do
    lib="$R/3360-ray-tracer_amd/librtx.so"; [ $v != product ] && lib="$R/3360-ray-tracer_amd/variants/librtx_$v.so"
    for a in "--workload c3_bunny --schedule park" "--adaptive --workload c3_bunny --schedule park" "--workload c2_final"; do
      RTX_LIB=$lib timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-generic-leg --no-adaptive-leg > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', '$a', round(d['value'],1), round(d['ms_per_step'],3), 'launch', round(d['roofline'].get('avg_launch_ms',0),3))"
    done
  done
done
