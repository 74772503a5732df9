#!/bin/bash
# Round 5 (r8e/r8f): record with the Markstein division by the sample count, then (r8f) the
# window replayed in one straight-line pass; A/B of the record window after the first phase
# (8 / 16) and of the phase floor (2^23 / 2^20), kernel traces.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
B="--adaptive --no-cpu-baseline --no-generic-leg --schedule park"
for r in 1 2; do
  for t in "rec_win=16" "rec_win=8" "phase_slots=1048576,rec_win=16" "phase_slots=1048576,rec_win=8"; do
    timeout -k 10 200 python bench.py $B --adapt-tune $t > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('$t', round(d['value'],1), round(d['ms_per_step'],3), 'traced', round(d['traced_value'],1))"
  done
done
export TMPDIR=/tmp
cd /tmp || exit 1
for w in 16 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/trace$w" -o run --output-format csv -- python3 "$R/bench.py" $B --adapt-tune phase_slots=1048576,rec_win=$w > "$R/$O/trace_bench$w.json" 2> "$R/$O/trace$w.err" || exit 1
done
echo traced
