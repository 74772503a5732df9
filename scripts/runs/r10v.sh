#!/bin/bash
# Round 6 (r10v): the adaptive first pass (min_spp samples of every pixel) on the fixed-spp kernel
# (first_map=0: per-wave 512 / 256-slot chunks) instead of the phase kernel (block-shared chunks),
# re-checked on the final build; C3 and C2 adaptive, interleaved.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r10v; mkdir -p $O
B="--adaptive --no-generic-leg --no-adaptive-leg --no-cpu-baseline"
: > $O/ab_first_map.txt
for r in 1 2; do
  for w in c3_bunny c2_final; do
    for fm in 1 0; do
      timeout -k 10 300 python bench.py $B --workload $w --adapt-tune first_map=$fm > $O/${w}_fm${fm}_$r.json 2> $O/${w}_fm${fm}_$r.err || { tail -5 $O/${w}_fm${fm}_$r.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/${w}_fm${fm}_$r.json').read().strip().splitlines()[-1]); print('round $r $w first_map=$fm', round(d['value'],1), round(d['ms_per_step'],3))" >> $O/ab_first_map.txt
    done
  done
done
cat $O/ab_first_map.txt
echo done
