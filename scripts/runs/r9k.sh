#!/bin/bash
# Round 5 (r9k): the early output at npix / 32 (variant ed32, r9j: C3 adaptive +0.7 %) on the 4K
# adaptive frame (C4), where the framebuffer copy is 15x longer; two interleaved rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r9k; mkdir -p $O
for r in 1 2; do
  for v in product ed32; do
    lib="$R/3360-ray-tracer_amd/librtx.so"; [ $v != product ] && lib="$R/3360-ray-tracer_amd/variants/librtx_$v.so"
    for a in "--adaptive --workload c4_bunny4k"; do
      RTX_LIB=$lib timeout -k 10 300 python bench.py $a --no-cpu-baseline --no-generic-leg --no-adaptive-leg > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', '$a', round(d['value'],1), round(d['ms_per_step'],3))"
    done
  done
done
