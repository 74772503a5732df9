#!/bin/bash
# Round 5 (r9b): guided slot claims in the fixed-spp kernel (the chunk = what the wave's last claim
# left of its region >> G, 64..512; variants g9 / g10 / g11) against the fixed 512-slot chunk.
# Parity subset on g10, then C3 at 16 and 200 spp and C2, two interleaved rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r9b; mkdir -p $O
RTX_LIB=$R/3360-ray-tracer_amd/variants/librtx_g10.so timeout -k 10 600 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_parity.py -m gpu -x -q -k "bunny or c3 or schedule or final" --timeout 300 --timeout-method thread > $O/pytest_g10.log 2>&1 || { tail -30 $O/pytest_g10.log; exit 1; }
tail -1 $O/pytest_g10.log
for r in 1 2; do
  for v in product g9 g10 g11; do
    lib="$R/3360-ray-tracer_amd/librtx.so"; [ $v != product ] && lib="$R/3360-ray-tracer_amd/variants/librtx_$v.so"
    for a in "--workload c3_bunny --spp 16" "--workload c3_bunny" "--workload c2_final"; do
      RTX_LIB=$lib timeout -k 10 200 python bench.py $a --schedule park --no-cpu-baseline --no-generic-leg --no-adaptive-leg > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', '$a', round(d['value'],1), round(d['ms_per_step'],3), 'launch', round(d['roofline']['avg_launch_ms'],3))"
    done
  done
done
