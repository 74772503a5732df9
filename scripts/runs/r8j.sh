#!/bin/bash
# Round 5 (r8j): the next batch from the prediction pooled over each pixel's 3 x 3 neighbourhood
# (k_adapt_plan) and the first margin, as ranked by scripts/adaptive_sim.py: adaptive GPU tests,
# then two interleaved rounds of the policy variants on C3 adaptive.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_parity.py -m gpu -x -q -k adaptive --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
B="--adaptive --no-cpu-baseline --no-generic-leg --schedule park"
for r in 1 2; do
  for t in "phase_slots=1048576" "phase_slots=2097152,margin1=0.8" "phase_slots=2097152,margin1=0.8,pool_w=8" "phase_slots=1048576,margin1=0.8,pool_w=8" "phase_slots=1048576,pool_w=3"; do
    timeout -k 10 200 python bench.py $B --adapt-tune $t > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('$t', round(d['value'],1), round(d['ms_per_step'],3), 'traced', round(d['traced_value'],1))"
  done
done
for t in "phase_slots=2097152,margin1=0.8,pool_w=8"; do
  RTX_DEBUG_ADAPT=1 timeout -k 10 120 python bench.py $B --steps 1 --warmup 1 --adapt-tune $t > $O/dbg.json 2> $O/dbg.err || { tail -20 $O/dbg.err; exit 1; }
  echo "== $t"; grep "rtx adaptive" $O/dbg.err | grep -v timeline | tail -4
done
