#!/bin/bash
# rocprofv3 passes for one bench configuration: kernel trace + stats, then PMC counters in
# separate passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline "$@" > "$OUT/bench_trace.json" 2> "$OUT/trace.err" || exit $?
for c in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM" \
         "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64"; do
  n=$(echo $c | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $c -d "$OUT/pmc_$n" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --steps 1 --warmup 0 "$@" > "$OUT/bench_pmc_$n.json" 2> "$OUT/pmc_$n.err" || exit $?
done
