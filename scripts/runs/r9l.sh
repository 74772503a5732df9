#!/bin/bash
# Round 5 (r9l): the final build (non-temporal records, PARK refill 12, early output at npix / 32): GPU suite, smoke, default bench line,
# C2 line, and the 2-rank rehearsal of the N > 1 path on one GPU (C4, 32 spp).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r9l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); a=d['adaptive']
print('default', round(d['value'],1), round(d['ms_per_step'],3), 'adaptive', round(a['value'],1), round(a['ms_per_step'],3), 'cpu', d['cpu_baseline']['value'])"
timeout -k 10 400 python bench.py --workload c2_final > $O/bench_c2_final.json 2> $O/bench_c2_final.err || { tail -20 $O/bench_c2_final.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_c2_final.json').read().strip().splitlines()[-1]); a=d['adaptive']
print('c2', round(d['value'],1), round(d['ms_per_step'],3), 'adaptive', round(a['value'],1), round(a['ms_per_step'],3))"
timeout -k 10 400 python bench.py --workload c4_bunny4k > $O/bench_c4_bunny4k.json 2> $O/bench_c4_bunny4k.err || { tail -20 $O/bench_c4_bunny4k.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_c4_bunny4k.json').read().strip().splitlines()[-1]); a=d['adaptive']
print('c4', round(d['value'],1), round(d['ms_per_step'],3), 'adaptive', round(a['value'],1), round(a['ms_per_step'],3))"
NPROC=2 timeout -k 10 500 bash scripts/multirank_rehearsal.sh --spp 32 || { tail -20 gpurun_out/bench_rehearsal_2rank.err; exit 1; }
cp gpurun_out/bench_rehearsal_2rank.json $O/
tail -1 $O/bench_rehearsal_2rank.json | cut -c1-300
