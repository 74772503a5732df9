#!/bin/bash
# Round 4: adaptive phases with block-shared slot chunks (MAP 1), the first pass on the phase
# kernel: parity, timeline, A/B of the first pass's kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5q; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_timed.py \
  -k "adaptive" > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
RTX_DEBUG_DRAIN=1 RTX_DEBUG_ADAPT=1 timeout -k 10 300 python3 scripts/drain_timeline.py > $O/out.txt 2> $O/timeline.txt || { tail $O/timeline.txt; exit 1; }
grep -E "adaptive" $O/timeline.txt
for rep in 1 2; do
  for arm in 1 0; do
    timeout -k 10 200 python bench.py --adaptive --no-cpu-baseline --no-generic-leg --adapt-tune first_map=$arm > $O/c3a_fm${arm}_$rep.json 2> $O/c3a_fm${arm}_$rep.err || exit 1
    python3 scripts/sweep_summary.py "c3a first_map=$arm rep $rep" $O/c3a_fm${arm}_$rep.json | tee -a $O/ab.txt
  done
done
# the uniform-group launch with block-shared chunks (variant build) on fixed-spp C3 / C2
timeout -k 10 900 bash scripts/ab.sh r5q_shared0_c3 "--no-generic-leg --no-adaptive-leg --no-cpu-baseline" default 3360-ray-tracer_amd/variants/librtx_shared0.so > /dev/null || exit 1
cat gpurun_out/ab_r5q_shared0_c3.txt
