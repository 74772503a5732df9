#!/bin/bash
# Round 5 (r8x): the PARK threshold and the refill threshold of the adaptive phase launches
# (MAP 1) on their own (variants p12 / p24: park at 12 / 24 walking lanes; r24 / r8: refill at
# 24 / 8 idle lanes) against the product (16 / 16), C3 adaptive, two interleaved rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8x; mkdir -p $O
for r in 1 2; do
  for v in product p12 p24 r24 r8; do
    lib="$R/3360-ray-tracer_amd/librtx.so"; [ $v != product ] && lib="$R/3360-ray-tracer_amd/variants/librtx_$v.so"
    RTX_LIB=$lib timeout -k 10 200 python bench.py --adaptive --no-cpu-baseline --no-generic-leg --schedule park > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', round(d['value'],1), round(d['ms_per_step'],3), 'traced', round(d['traced_value'],1))"
  done
done
