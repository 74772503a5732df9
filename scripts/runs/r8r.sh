#!/bin/bash
# Round 5 (r8r): the adaptive policy on the 4K workloads: the default (pooled prediction, first
# margin 0.8, floor 2^21) against round 4's (own prediction, margin 1, floor 2^23) on C4 and C5.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8r; mkdir -p $O
for r in 1 2; do
  for w in c4_bunny4k c5_mixed; do
    for t in "pool_w=8" "phase_slots=8388608,margin1=1.0,pool_w=0"; do
      timeout -k 10 300 python bench.py --adaptive --workload $w --no-cpu-baseline --no-generic-leg --steps 3 --warmup 1 --adapt-tune $t > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
      python3 -c "
import json
d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('$w $t', round(d['value'],1), round(d['ms_per_step'],3), 'traced', round(d['traced_value'],1))"
    done
  done
done
