#!/bin/bash
# Round 4: the tile schedule with small tiles, many in flight, and the rest of the budget for
# the last pixels of a tile (fewer phase chains); lane occupancy of the tracing rounds; the phase
# schedule beside it; the reference's calibration with serial and with parallel shading.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5d; mkdir -p $O
B="--adaptive --steps 6 --warmup 1 --no-cpu-baseline --no-generic-leg"
run() {  # tag, extra args
  timeout -k 10 120 python bench.py $B $2 > $O/sweep_$1.json 2> $O/sweep_$1.err || exit 1
  python3 scripts/sweep_summary.py $1 $O/sweep_$1.json >> $O/sweep.txt
}
run phases "--adapt-schedule phases"
run fixed_c3 "--no-adaptive-leg"
run tp8 "--adapt-tune tile_tp=8"
for t in tile_tp=8,tile_nt=16,tile_tail=8,tile_kcap=200 tile_tp=8,tile_nt=16,tile_tail=8,tile_kcap=200,tile_margin=1.25 \
         tile_tp=8,tile_nt=16,tile_tail=4,tile_kcap=200 tile_tp=8,tile_nt=16,tile_tail=2,tile_kcap=200 \
         tile_tp=4,tile_nt=16 tile_tp=4,tile_nt=16,tile_tail=4,tile_kcap=200 tile_tp=2,tile_nt=16 \
         tile_tp=8,tile_nt=16,tile_kinc=16,tile_mstep=0.5 tile_tp=8,tile_nt=16,tile_margin=1.5,tile_kcap=200; do
  run "$t" "--adapt-tune $t"
done
cat $O/sweep.txt
timeout -k 10 300 python scripts/calibrate_cpu.py --threads 16 --serial-shading --host "GPU box host (MI355X pool), 16 threads" --out $O/cpu_calibration_16t_serial_shading.json > $O/calibrate_serial.log 2>&1 || exit 1
timeout -k 10 300 python scripts/calibrate_cpu.py --threads 16 --host "GPU box host (MI355X pool), 16 threads" --out $O/cpu_calibration_16t.json > $O/calibrate.log 2>&1 || exit 1
echo done
