#!/bin/bash
# Round 5 (r8l): the build with compacted phase lists, the Markstein record and the 2^20 phase
# floor: GPU suite, smoke, the default bench line, C2 / C4 / C5 bench lines (reference
# cpu_baseline), then stochastic PC sampling of the fixed-spp C3 frame.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); a=d['adaptive']
print('default', round(d['value'],1), round(d['ms_per_step'],3), 'adaptive', round(a['value'],1), round(a['ms_per_step'],3), 'cpu', d['cpu_baseline']['value'])"
for w in c2_final c4_bunny4k c5_mixed; do
  timeout -k 10 400 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_$w.json').read().strip().splitlines()[-1]); print('$w', round(d['value'],1), round(d['ms_per_step'],3), d['roofline'].get('frac'), d['cpu_baseline']['value'])"
done
exit 0
