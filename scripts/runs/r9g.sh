#!/bin/bash
# Round 5 (r9g): the PARK kernel's refill threshold, confirmation: kRefillMinPark 12 (r9f: adaptive
# +0.45 %, fixed +-0) and 10 / 14 against 16; C3 adaptive and fixed, three interleaved rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r9g; mkdir -p $O
for r in 1 2 3; do
  for v in product rf10 rf12 rf14; do
    lib="$R/3360-ray-tracer_amd/librtx.so"; [ $v != product ] && lib="$R/3360-ray-tracer_amd/variants/librtx_$v.so"
    for a in "--adaptive --workload c3_bunny" "--workload c3_bunny"; do
      RTX_LIB=$lib timeout -k 10 200 python bench.py $a --schedule park --no-cpu-baseline --no-generic-leg --no-adaptive-leg > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', '$a', round(d['value'],1), round(d['ms_per_step'],3))"
    done
  done
done
