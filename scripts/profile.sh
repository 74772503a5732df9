#!/bin/bash
# rocprofv3 passes for one bench configuration: kernel trace + stats, then PMC counters, one
# pass per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; at most
# 8 SQ / 4 TCC / 2 GRBM counters per pass).  Every pass runs under its own time limit.
#   scripts/profile.sh <tag> <bench args...>
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
B="--no-cpu-baseline --no-generic-leg --no-adaptive-leg"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" $B "$@" > "$OUT/bench_trace.json" 2> "$OUT/trace.err" || exit $?
# SQ_ACTIVE_INST_VALU2 (gfx950): quad-cycles in which a SIMD issued two VALU instructions, so
# the SIMD's VALU issue quad-cycles are SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2 (the
# microbenchmark scripts/microbench/valu_ceiling.hip checks this against measured cycles)
for c in FETCH_SIZE WRITE_SIZE \
         "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU" \
         "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32" \
         "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32"; do
  n=$(echo $c | cut -d' ' -f1-2 | tr ' ' '_')
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $c -d "$OUT/pmc_$n" -o run --output-format csv -- python3 "$R/bench.py" $B --steps 2 --warmup 1 "$@" > "$OUT/bench_pmc_$n.json" 2> "$OUT/pmc_$n.err" || exit $?
done
