#!/bin/bash
# Round 5 (r8d): compacted per-phase pixel lists (record / floor / scan / expand over the phase's
# pixels only; 16-sample record windows after the first phase): GPU suite, adaptive A/B of the
# phase floor (the schedule simulator, scripts/adaptive_sim.py, ranks 2^20 first), kernel trace.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
B="--adaptive --no-cpu-baseline --no-generic-leg --schedule park"
for r in 1 2; do
  for t in "" "phase_slots=1048576" "phase_slots=2097152" "phase_slots=4194304"; do
    timeout -k 10 200 python bench.py $B ${t:+--adapt-tune $t} > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('${t:-default}', round(d['value'],1), round(d['ms_per_step'],3), 'traced', round(d['traced_value'],1), 'hot', round(d['hot_kernel_ms_per_step'],3) if 'hot_kernel_ms_per_step' in d else None)"
  done
done
for t in "phase_slots=8388608" "phase_slots=1048576"; do
  RTX_DEBUG_ADAPT=1 timeout -k 10 120 python bench.py $B --steps 1 --warmup 1 --adapt-tune $t > $O/dbg.json 2> $O/dbg.err || { tail -20 $O/dbg.err; exit 1; }
  echo "== $t"; grep "rtx adaptive" $O/dbg.err | grep -v timeline | tail -6
done
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/trace" -o run --output-format csv -- python3 "$R/bench.py" $B > "$R/$O/trace_bench.json" 2> "$R/$O/trace.err" || exit 1
echo traced
