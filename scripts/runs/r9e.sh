#!/bin/bash
# Round 5 (r9e): the final build (non-temporal radiance records): C4 / C5 bench lines; the
# slot map read non-temporal in the phase launches (variant ntmap: parity subset, C3 adaptive and
# fixed, two interleaved rounds); then C3 fixed and C3 adaptive profiles (kernel trace + PMC
# passes, scripts/profile.sh) for the rooflines' sources.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r9e; mkdir -p $O
for w in c4_bunny4k c5_mixed; do
  timeout -k 10 400 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_$w.json').read().strip().splitlines()[-1]); a=d['adaptive']
print('$w', round(d['value'],1), round(d['ms_per_step'],3), 'adaptive', round(a['value'],1), round(a['ms_per_step'],3), d['roofline'].get('frac'), d['cpu_baseline']['value'])"
done
RTX_LIB=$R/3360-ray-tracer_amd/variants/librtx_ntmap.so timeout -k 10 600 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_parity.py -m gpu -x -q -k "bunny or c3 or schedule or final" --timeout 300 --timeout-method thread > $O/pytest_ntmap.log 2>&1 || { tail -30 $O/pytest_ntmap.log; exit 1; }
tail -1 $O/pytest_ntmap.log
for r in 1 2; do
  for v in product ntmap; do
    lib="$R/3360-ray-tracer_amd/librtx.so"; [ $v != product ] && lib="$R/3360-ray-tracer_amd/variants/librtx_$v.so"
    for a in "--adaptive --workload c3_bunny --schedule park" "--adaptive --workload c2_final"; do
      RTX_LIB=$lib timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-generic-leg --no-adaptive-leg > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', '$a', round(d['value'],1), round(d['ms_per_step'],3))"
    done
  done
done
timeout -k 10 600 bash scripts/profile.sh r9e_c3 --workload c3_bunny --schedule park || exit 1
echo "c3 profiled"
timeout -k 10 600 bash scripts/profile.sh r9e_c3a --adaptive --workload c3_bunny --schedule park || exit 1
echo "c3a profiled"
