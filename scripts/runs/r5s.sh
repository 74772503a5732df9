#!/bin/bash
# Round 4, final build: GPU suite, smoke, the default bench line, C3 adaptive profile (the
# adaptive roofline's PMC source), the 2-rank rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5s; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -5 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
python3 scripts/sweep_summary.py default $O/bench_default.json
timeout -k 10 700 bash scripts/profile.sh r5s_c3a --schedule park --adaptive || exit 1
echo "c3a profiled"
NPROC=2 timeout -k 10 450 bash scripts/multirank_rehearsal.sh || exit 1
cp gpurun_out/bench_rehearsal_2rank.json gpurun_out/bench_rehearsal_2rank.err $O/
echo done
