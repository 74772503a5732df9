#!/bin/bash
# Round 5 (r8g): where k_adapt_record's time goes: kernel traces of the record with its replay
# compiled out (fetch only) and with its loads compiled out (replay of whatever LDS holds)
# against the product build (A/B variant builds; their pixels are wrong by construction).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8g; mkdir -p $O
export TMPDIR=/tmp
cd /tmp || exit 1
B="--adaptive --no-cpu-baseline --no-generic-leg --schedule park --steps 3 --warmup 1 --adapt-tune phase_slots=1048576,rec_win=8"
for v in product rec_nocompute rec_nofetch; do
  lib="$R/3360-ray-tracer_amd/librtx.so"; [ $v != product ] && lib="$R/3360-ray-tracer_amd/variants/librtx_$v.so"
  RTX_LIB=$lib timeout -k 10 100 rocprofv3 --kernel-trace --stats -d "$R/$O/trace_$v" -o run --output-format csv -- python3 "$R/bench.py" $B > "$R/$O/bench_$v.json" 2> "$R/$O/bench_$v.err"
  rc=$?
  echo "$v rc=$rc"
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit 1
done
exit 0
