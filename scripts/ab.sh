#!/bin/bash
# A/B variant libraries in ONE process-sequence on one GPU:
#   bash scripts/ab.sh TAG "bench args" lib1.so lib2.so ...   (default lib = product)
# Interleaves rounds (lib1, lib2, ..., lib1, lib2, ...) so DVFS/thermal drift hits all.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" || exit 1
mkdir -p gpurun_out
TAG=$1; shift
ARGS=$1; shift
OUT=gpurun_out/ab_$TAG.txt
: > $OUT
for round in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = "default" ]; then L=""; else L="$R/$lib"; fi
    res=$(RTX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline $ARGS 2>>gpurun_out/ab_$TAG.err) || exit $?
    echo "round $round $lib $(echo "$res" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d["roofline"]; print("%.1f Mrays/s ms/step %.2f frac %s nodes/seg %.3f prims/seg %.3f" % (d["value"], d["ms_per_step"], r.get("frac"), r.get("nodes_per_segment", 0), r.get("prims_per_segment", 0)))')" >> $OUT
  done
done
cat $OUT
