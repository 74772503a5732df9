#!/bin/bash
# Round 5 (r8i): the generic kernel builds (RTX_FLAG_GENERIC: every primitive kind, material and
# texture path; 32 VGPRs spilled at 4 waves per SIMD) at 3 waves per SIMD (no spills): A/B of
# the generic leg on C3 and C2, two interleaved rounds (variant build gw3).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8i; mkdir -p $O
for r in 1 2; do
  for v in product gw3; do
    lib="$R/3360-ray-tracer_amd/librtx.so"; [ $v != product ] && lib="$R/3360-ray-tracer_amd/variants/librtx_$v.so"
    for w in c3_bunny c2_final; do
      RTX_LIB=$lib timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-adaptive-leg > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); g=d['generic_build']
print('$v $w', round(d['value'],1), 'generic', round(g['value'],1), round(g['value']/d['value'],3))"
    done
  done
done
