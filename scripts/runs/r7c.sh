#!/bin/bash
# Round 5: carried paths + a last phase that drains with full budgets — GPU suite, debug lines,
# C3 adaptive A/B over the last phase's size and against draining every launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r7c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
B="--adaptive --no-cpu-baseline --no-generic-leg --schedule park"
RTX_DEBUG_ADAPT=1 timeout -k 10 120 python bench.py $B --steps 1 --warmup 1 > $O/debug_carry.json 2> $O/debug_carry.err || exit 1
grep "rtx adaptive" $O/debug_carry.err | grep -v timeline | tail -8
for r in 1 2; do
  for t in "carry=1" "carry=1,final_slots=8388608" "carry=1,final_slots=25165824" "carry=1,final_slots=50331648" "carry=0"; do
    timeout -k 10 200 python bench.py $B --adapt-tune $t > $O/ab.json 2> $O/ab.err || exit 1
    python3 -c "
import json
d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('$t', round(d['value'],1), round(d['ms_per_step'],3), 'traced', round(d['traced_value'],1), 'launches', d['roofline'].get('avg_launch_ms'))"
  done
done
