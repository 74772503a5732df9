#!/bin/bash
# Round 5 (r8o): host waits that spin on the pinned count / statistics word before taking the
# event, against the previous build (variants/librtx_prev.so): adaptive C3 and fixed C3 / C2,
# two interleaved rounds; host timestamps of the new build.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8o; mkdir -p $O
for r in 1 2; do
  for v in prev spin; do
    lib="$R/3360-ray-tracer_amd/librtx.so"; [ $v = prev ] && lib="$R/3360-ray-tracer_amd/variants/librtx_prev.so"
    for a in "--adaptive --workload c3_bunny" "--workload c3_bunny" "--workload c2_final" "--adaptive --workload c2_final"; do
      RTX_LIB=$lib timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-generic-leg --no-adaptive-leg > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', '$a', round(d['value'],1), round(d['ms_per_step'],3))"
    done
  done
done
RTX_DEBUG_HOST=1 timeout -k 10 120 python3 bench.py --adaptive --no-cpu-baseline --no-generic-leg --schedule park --steps 20 > $O/host.json 2> $O/host.err || exit 1
grep "rtx host" $O/host.err | tail -3
