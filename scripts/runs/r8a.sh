#!/bin/bash
# Round 5 (r8a): the build without carried paths: the whole GPU suite (with the whole-frame
# parity tests), smoke, the default bench line (reference cpu_baseline), then the C3 adaptive
# and C2 profiles with the dual-issue counter groups.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json
timeout -k 10 900 bash scripts/profile.sh r8a_c3a --adaptive || exit 1
echo "c3a profiled"
timeout -k 10 900 bash scripts/profile.sh r8a_c2 --workload c2_final || exit 1
echo "c2 profiled"
