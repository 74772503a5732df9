#!/bin/bash
# Round 5 (r8b): k_adapt_record with LDS-transposed windows and spread pixel counters (no
# same-address atomics in record / expand): the GPU suite, the adaptive bench line and its
# kernel trace, then the C2 / C3-adaptive / C4 / C5 profiles with the schedule forced (so the
# schedule-timing launches of a first render stay out of the PMC sums).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --adaptive --no-cpu-baseline --no-generic-leg --schedule park > $O/bench_c3a_$r.json 2> $O/bench_c3a_$r.err || { tail -20 $O/bench_c3a_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_c3a_$r.json').read().strip().splitlines()[-1]); print('c3a', round(d['value'],1), round(d['ms_per_step'],3), 'traced', round(d['traced_value'],1))"
done
timeout -k 10 900 bash scripts/profile.sh r8b_c3a --adaptive --schedule park || exit 1
echo "c3a profiled"
timeout -k 10 900 bash scripts/profile.sh r8b_c2 --workload c2_final --schedule plain || exit 1
echo "c2 profiled"
timeout -k 10 900 bash scripts/profile.sh r8b_c4 --workload c4_bunny4k --schedule park || exit 1
echo "c4 profiled"
timeout -k 10 900 bash scripts/profile.sh r8b_c5 --workload c5_mixed --schedule plain || exit 1
echo "c5 profiled"
