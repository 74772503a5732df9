#!/bin/bash
# Round 4, first GPU call: the adaptive tile schedule's parity tests, C3 adaptive with the tile
# schedule (first pass in a launch of its own / inside the tile launch) and the phase schedule
# (bench lines + one debug frame each: per-launch times), then the timed adaptive oracle tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "adaptive_schedules or group_size or persistent_schedule_equals or stripes" > $O/pytest_parity.log 2>&1 || exit 1
B="--adaptive --steps 10 --warmup 2 --no-cpu-baseline --no-generic-leg"
timeout -k 10 120 python bench.py $B > $O/bench_c3a_tiles.json 2> $O/bench_c3a_tiles.err || exit 1
timeout -k 10 120 python bench.py $B --adapt-tune tile_first_pass=1 > $O/bench_c3a_tiles1.json 2> $O/bench_c3a_tiles1.err || exit 1
timeout -k 10 120 python bench.py $B --adapt-schedule phases > $O/bench_c3a_phases.json 2> $O/bench_c3a_phases.err || exit 1
D="--adaptive --steps 1 --warmup 1 --no-cpu-baseline --no-generic-leg"
RTX_DEBUG_ADAPT=1 timeout -k 10 120 python bench.py $D > $O/dbg_tiles.json 2> $O/dbg_tiles.err || exit 1
RTX_DEBUG_ADAPT=1 timeout -k 10 120 python bench.py $D --adapt-tune tile_first_pass=1 > $O/dbg_tiles1.json 2> $O/dbg_tiles1.err || exit 1
RTX_DEBUG_ADAPT=1 timeout -k 10 120 python bench.py $D --adapt-schedule phases > $O/dbg_phases.json 2> $O/dbg_phases.err || exit 1
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_timed.py \
  -k "adaptive" > $O/pytest_timed.log 2>&1 || exit 1
echo done
