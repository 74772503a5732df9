#!/bin/bash
# Round 4: the tile schedule with the idle-aware batch margin (starve gain) on C3 adaptive.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5e; mkdir -p $O
B="--adaptive --steps 6 --warmup 1 --no-cpu-baseline --no-generic-leg"
run() {  # tag, extra args
  timeout -k 10 120 python bench.py $B $2 > $O/sweep_$1.json 2> $O/sweep_$1.err || exit 1
  python3 scripts/sweep_summary.py $1 $O/sweep_$1.json >> $O/sweep.txt
}
run phases "--adapt-schedule phases"
for t in tile_tp=8 tile_tp=8,tile_nt=16 tile_tp=8,tile_starve=0.25 tile_tp=8,tile_starve=0.5 tile_tp=8,tile_starve=1 \
         tile_tp=8,tile_nt=16,tile_starve=0.5 tile_tp=8,tile_nt=16,tile_starve=1,tile_kcap=200 \
         tile_tp=8,tile_starve=2,tile_kcap=200 tile_tp=16,tile_starve=1,tile_kcap=200 tile_tp=4,tile_nt=16,tile_starve=1; do
  run "$t" "--adapt-tune $t"
done
cat $O/sweep.txt
echo done
