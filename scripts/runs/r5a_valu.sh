#!/bin/bash
# Round 5: VALU issue-cost microbenchmark (stamps + HIP events), then one PMC pass over it.
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out"
timeout -k 10 180 "$R/scripts/microbench/valu_ceiling" > "$R/gpurun_out/valu_ceiling.jsonl" 2> "$R/gpurun_out/valu_ceiling.err" || exit $?
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d "$R/gpurun_out/valu_pmc" -o run --output-format csv -- "$R/scripts/microbench/valu_ceiling" 1024 > "$R/gpurun_out/valu_ceiling_pmc.jsonl" 2> "$R/gpurun_out/valu_pmc.err" || exit $?
cd "$R" && timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/bench_r5a.json 2> gpurun_out/bench_r5a.err
