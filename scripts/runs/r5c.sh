#!/bin/bash
# Round 4: the tile schedule's knobs on C3 adaptive (one bench line each: value, traced, idle
# wave rounds), then the A/Bs of r5b (quantised nodes, camera-only refill) and the CPU
# calibration of the reference with its parallel shading loop on this host.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5c; mkdir -p $O
B="--adaptive --steps 6 --warmup 1 --no-cpu-baseline --no-generic-leg"
for t in default tile_tp=16 tile_tp=8 tile_nt=16 tile_tp=16,tile_nt=16 tile_tp=8,tile_nt=16 tile_kinc=16 \
         tile_margin=1.25 tile_mstep=0.25 tile_tail=4 tile_tail=12 tile_kcap=200 tile_first_pass=1 \
         tile_first_pass=1,tile_tp=16,tile_nt=16; do
  a=""; [ "$t" != default ] && a="--adapt-tune $t"
  timeout -k 10 120 python bench.py $B $a > $O/sweep_$t.json 2> $O/sweep_$t.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$O/sweep_$t.json').read().strip().splitlines()[-1]); print('$t', round(d['value'],1), round(d['traced_value'],1), round(d['ms_per_step'],2), d['roofline'].get('wave_rounds_idle_frac'))" >> $O/sweep.txt
done
cat $O/sweep.txt
RTX_LIB=$PWD/3360-ray-tracer_amd/variants/librtx_qnode.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "fast_matches_parity or persistent_schedule_equals or parked_traversal" > $O/pytest_qnode.log 2>&1 || exit 1
timeout -k 10 600 bash scripts/ab.sh r5c_qnode_c3 "--no-generic-leg --no-adaptive-leg" default 3360-ray-tracer_amd/variants/librtx_qnode.so > /dev/null || exit 1
timeout -k 10 600 bash scripts/ab.sh r5c_camkarg_c3 "--no-generic-leg --no-adaptive-leg" default 3360-ray-tracer_amd/variants/librtx_camkarg.so > /dev/null || exit 1
timeout -k 10 300 python scripts/calibrate_cpu.py --threads 16 --host "GPU box host (MI355X pool), 16 threads" --out $O/cpu_calibration_16t.json > $O/calibrate.log 2>&1 || exit 1
echo done
