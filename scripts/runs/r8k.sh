#!/bin/bash
# Round 5 (r8k): adaptive policy A/B on C3 and C2 (scripts/adaptive_sim.py's joint ranking):
# pooled prediction + first margin 0.8 + floor 2^21, with and without finishing every pixel in
# the next phase when that costs fewer than 2^22 extra slots, against the current default.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_parity.py -m gpu -x -q -k adaptive --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
B="--adaptive --no-cpu-baseline --no-generic-leg"
for r in 1 2; do
  for w in c3_bunny c2_final; do
    for t in "phase_slots=1048576" "phase_slots=2097152,margin1=0.8,pool_w=8" "phase_slots=2097152,margin1=0.8,pool_w=8,finish_slots=4194304" "phase_slots=8388608,margin1=0.8,pool_w=8,finish_slots=4194304"; do
      timeout -k 10 200 python bench.py $B --workload $w --adapt-tune $t > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
      python3 -c "
import json
d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('$w $t', round(d['value'],1), round(d['ms_per_step'],3), 'traced', round(d['traced_value'],1))"
    done
  done
done
