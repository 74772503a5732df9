#!/bin/bash
# Round 5 (r7f: blocked pixels without a smallest batch): carried-path variants with the prediction over all ended samples on C3 adaptive (which launches carry, blocked pixels held,
# the last phase's size) against draining every launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r7f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k adaptive --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
B="--adaptive --no-cpu-baseline --no-generic-leg --schedule park"
for r in 1 2; do
  for t in "carry=1" "carry=1,carry_until=2" "carry=1,final_slots=25165824" "carry=1,phase_slots=4194304" "carry=0"; do
    timeout -k 10 200 python bench.py $B --adapt-tune $t > $O/ab.json 2> $O/ab.err || exit 1
    python3 -c "
import json
d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('$t', round(d['value'],1), round(d['ms_per_step'],3), 'traced', round(d['traced_value'],1), 'launches', d['roofline'].get('avg_launch_ms'))"
  done
done
for t in "carry=1" "carry=0"; do
  RTX_DEBUG_ADAPT=1 timeout -k 10 120 python bench.py $B --steps 1 --warmup 1 --adapt-tune $t > $O/dbg.json 2> $O/dbg.err || exit 1
  echo "== $t"; grep "rtx adaptive" $O/dbg.err | grep -v timeline | head -6
done
