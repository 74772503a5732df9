#!/bin/bash
# Round 5 (r8q): the speculative walk prefetching the node it will pop next (global_load_lds of
# one dword of its line into a scratch LDS row) when a visit pushes children: variant build pf
# against the product; parity subset on the variant, then C3 fixed / adaptive A/B (two rounds).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8q; mkdir -p $O
RTX_LIB=$R/3360-ray-tracer_amd/variants/librtx_pf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_timed.py -m gpu -x -q -k "c3 or bunny" --timeout 300 --timeout-method thread > $O/pytest_pf.log 2>&1 || { tail -30 $O/pytest_pf.log; exit 1; }
tail -1 $O/pytest_pf.log
for r in 1 2; do
  for v in product pf; do
    lib="$R/3360-ray-tracer_amd/librtx.so"; [ $v = pf ] && lib="$R/3360-ray-tracer_amd/variants/librtx_pf.so"
    for a in "--workload c3_bunny" "--adaptive --workload c3_bunny"; do
      RTX_LIB=$lib timeout -k 10 200 python bench.py $a --schedule park --no-cpu-baseline --no-generic-leg --no-adaptive-leg > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', '$a', round(d['value'],1), round(d['ms_per_step'],3))"
    done
  done
done
