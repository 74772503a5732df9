#!/bin/bash
# Round 5: the VALU microbenchmark's remaining classes and its PMC pass with the dual-issue
# counter (SQ_ACTIVE_INST_VALU2), then the C3 profile of the current build with it.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r7a; mkdir -p $O
timeout -k 10 180 scripts/microbench/valu_ceiling 2048 12 > $O/valu_ceiling_b.jsonl 2> $O/valu_ceiling_b.err || exit 1
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d "$R/$O/valu_pmc" -o run --output-format csv -- "$R/scripts/microbench/valu_ceiling" 1024 > "$R/$O/valu_ceiling_pmc.jsonl" 2> "$R/$O/valu_pmc.err" ) || exit 1
echo "microbench done"
timeout -k 10 900 bash scripts/profile.sh r7a_c3 --schedule park || exit 1
echo "c3 profiled"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -5 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
