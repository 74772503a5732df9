#!/bin/bash
# Round 4: the tile launch's timeline (counting build: when blocks find the claim order used up,
# when waves end) for a few settings of the pipelined tile schedule.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5g; mkdir -p $O
D="--adaptive --steps 1 --warmup 1 --no-cpu-baseline --no-generic-leg"
for t in default tile_split=1000000 tile_nt=4 tile_tp=4 tile_tp=16,tile_nt=4 tile_starve=1,tile_kinc=16; do
  a=""; [ "$t" != default ] && a="--adapt-tune $t"
  RTX_DEBUG_ADAPT=1 timeout -k 10 120 python bench.py $D $a > $O/dbg_$t.json 2> $O/dbg_$t.err || exit 1
  echo "== $t" >> $O/timeline.txt; grep "rtx adaptive" $O/dbg_$t.err | tail -3 >> $O/timeline.txt
done
cat $O/timeline.txt
