#!/bin/bash
# Round 5 (r9f): the PARK kernel's park threshold (kParkAt 12 / 20) and refill threshold
# (kRefillMinPark 12 / 20) against 16 / 16, re-checked with the non-temporal records; C3 fixed and
# adaptive, two interleaved rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r9f; mkdir -p $O
for r in 1 2; do
  for v in product pa12 pa20 rf12 rf20; do
    lib="$R/3360-ray-tracer_amd/librtx.so"; [ $v != product ] && lib="$R/3360-ray-tracer_amd/variants/librtx_$v.so"
    for a in "--workload c3_bunny" "--adaptive --workload c3_bunny"; do
      RTX_LIB=$lib timeout -k 10 200 python bench.py $a --schedule park --no-cpu-baseline --no-generic-leg --no-adaptive-leg > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', '$a', round(d['value'],1), round(d['ms_per_step'],3))"
    done
  done
done
