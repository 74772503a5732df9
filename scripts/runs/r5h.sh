#!/bin/bash
# Round 4: the tile schedule with eagerly laid out front/back batches and the record's statistics
# in LDS: parity, then C3 adaptive sweeps beside the phase schedule, the timeline, full budget.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5h; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 60 --timeout-method thread tests/test_gpu_parity.py \
  -k "adaptive_schedules or group_size or persistent_schedule_equals" > $O/pytest_parity.log 2>&1 || exit 1
B="--adaptive --steps 6 --warmup 1 --no-cpu-baseline --no-generic-leg"
run() {  # tag, extra args
  timeout -k 10 120 python bench.py $B $2 > $O/sweep_$1.json 2> $O/sweep_$1.err || exit 1
  python3 scripts/sweep_summary.py $1 $O/sweep_$1.json >> $O/sweep.txt
}
run phases "--adapt-schedule phases"
run default ""
for t in tile_nt=10 tile_nt=4 tile_tp=4 tile_split=16 tile_split=1000000 tile_tail=2 tile_kinc=16; do
  run "$t" "--adapt-tune $t"
done
cat $O/sweep.txt
RTX_DEBUG_ADAPT=1 timeout -k 10 120 python bench.py --adaptive --steps 1 --warmup 1 --no-cpu-baseline \
  --no-generic-leg > $O/dbg.json 2> $O/dbg.err || exit 1
grep "rtx adaptive" $O/dbg.err | tail -4
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_timed.py \
  -k "adaptive" > $O/pytest_timed.log 2>&1 || exit 1
echo done
