#!/bin/bash
# Round 5 (r8t): the final build: GPU suite, smoke, default bench line, and the C3 adaptive
# profile (PMC passes over every phase launch) for the adaptive roofline's source.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8t; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); a=d['adaptive']
print('default', round(d['value'],1), round(d['ms_per_step'],3), 'adaptive', round(a['value'],1), round(a['ms_per_step'],3), 'cpu', d['cpu_baseline']['value'])"
timeout -k 10 900 bash scripts/profile.sh r8t_c3a --adaptive --schedule park || exit 1
echo "c3a profiled"
