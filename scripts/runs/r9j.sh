#!/bin/bash
# Round 5 (r9j): the adaptive early output's start: once a phase holds <= npix / 8 or / 32 pixels
# (variants ed8 / ed32) instead of / 4 (a later copy, a smaller device patch); C3 and C2 adaptive,
# two interleaved rounds, after the early-output test on ed8.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r9j; mkdir -p $O
RTX_LIB=$R/3360-ray-tracer_amd/variants/librtx_ed8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_timed.py -m gpu -x -q -k "early_output or whole_frame" --timeout 200 --timeout-method thread > $O/pytest_ed8.log 2>&1 || { tail -30 $O/pytest_ed8.log; exit 1; }
tail -1 $O/pytest_ed8.log
for r in 1 2; do
  for v in product ed8 ed32; do
    lib="$R/3360-ray-tracer_amd/librtx.so"; [ $v != product ] && lib="$R/3360-ray-tracer_amd/variants/librtx_$v.so"
    for a in "--adaptive --workload c3_bunny --schedule park" "--adaptive --workload c2_final"; do
      RTX_LIB=$lib timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-generic-leg --no-adaptive-leg > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', '$a', round(d['value'],1), round(d['ms_per_step'],3))"
    done
  done
done
