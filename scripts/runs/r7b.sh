#!/bin/bash
# Round 5: carried paths across adaptive phase launches — GPU suite, per-phase debug lines,
# C3 adaptive A/B (carry on / off), default line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r7b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
B="--adaptive --no-cpu-baseline --no-generic-leg --schedule park"
RTX_DEBUG_ADAPT=1 timeout -k 10 120 python bench.py $B --steps 1 --warmup 1 > $O/debug_carry.json 2> $O/debug_carry.err || exit 1
RTX_DEBUG_ADAPT=1 timeout -k 10 120 python bench.py $B --steps 1 --warmup 1 --adapt-tune carry=0 > $O/debug_drain.json 2> $O/debug_drain.err || exit 1
grep "rtx adaptive" $O/debug_carry.err | tail -12
grep "rtx adaptive" $O/debug_drain.err | tail -6
for r in 1 2; do
  timeout -k 10 200 python bench.py $B > $O/ab_carry_$r.json 2> $O/ab_carry_$r.err || exit 1
  timeout -k 10 200 python bench.py $B --adapt-tune carry=0 > $O/ab_drain_$r.json 2> $O/ab_drain_$r.err || exit 1
  python3 -c "
import json
for k in ('carry','drain'):
    d=json.loads(open('$O/ab_'+k+'_$r.json').read().strip().splitlines()[-1]); print(k, round(d['value'],1), round(d['ms_per_step'],3), 'traced', round(d['traced_value'],1))"
done
