#!/bin/bash
# Round 5 (r8s): cost of write-through (sc0 sc1) radiance-record stores in the hot kernel, the
# precondition of an in-launch hand-off of finished bands to the accumulate: variant wt against
# the product, C3 / C2 fixed, two interleaved rounds (pixels unchanged: only the store policy).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8s; mkdir -p $O
for r in 1 2; do
  for v in product wt; do
    lib="$R/3360-ray-tracer_amd/librtx.so"; [ $v = wt ] && lib="$R/3360-ray-tracer_amd/variants/librtx_wt.so"
    for w in c3_bunny c2_final; do
      RTX_LIB=$lib timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-generic-leg --no-adaptive-leg > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v $w', round(d['value'],1), round(d['ms_per_step'],3), 'launch', round(d['roofline']['avg_launch_ms'],3), 'rms', d.get('rms_vs_cpu'))"
    done
  done
done
