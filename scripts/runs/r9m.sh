#!/bin/bash
# Round 5 (r9m): the adaptive launches' block-shared slot chunk (kChunkShared 128) at 64 / 192,
# re-checked on the final build; C3 and C2 adaptive, two interleaved rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r9m; mkdir -p $O
for r in 1 2; do
  for v in product cs64 cs192; do
    lib="$R/3360-ray-tracer_amd/librtx.so"; [ $v != product ] && lib="$R/3360-ray-tracer_amd/variants/librtx_$v.so"
    for a in "--adaptive --workload c3_bunny --schedule park" "--adaptive --workload c2_final"; do
      RTX_LIB=$lib timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-generic-leg --no-adaptive-leg > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', '$a', round(d['value'],1), round(d['ms_per_step'],3))"
    done
  done
done
