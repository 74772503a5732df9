#!/bin/bash
# Per-kernel device times of variant libraries (rocprofv3 --kernel-trace --stats, one run each):
#   bash scripts/prof_ab.sh TAG "bench args" lib1.so lib2.so ...   ("default" = the product)
# Writes gpurun_out/profab_<TAG>.txt: lib, kernel, calls, average ns.
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
ARGS=$1; shift
OUT="$R/gpurun_out/profab_$TAG.txt"
mkdir -p "$R/gpurun_out"
: > "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
for lib in "$@"; do
  if [ "$lib" = "default" ]; then L=""; else L="$R/$lib"; fi
  D="$R/gpurun_out/profab_${TAG}_$(basename "$lib" .so)"
  RTX_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$D" -o run --output-format csv -- \
    python3 "$R/bench.py" --no-cpu-baseline $ARGS > "$D.json" 2> "$D.err" || exit $?
  python3 - "$D" "$lib" >> "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/*kernel_stats.csv")[0]
for r in csv.DictReader(open(f)):
    print("%-28s %-70s %5s %12.1f" % (sys.argv[2].split("/")[-1], r["Name"][:70], r["Calls"], float(r["AverageNs"])))
PY
done
cat "$OUT"
