#!/bin/bash
# Round 5 (r8y): the restated small-argument cos / sin (kSincosSmall) in the PARK TU too (variant
# sc; 3 VGPRs spilled now, against 10-19 when round 2 / 3 measured it): parity subset on the
# variant, then C3 fixed and adaptive, two interleaved rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8y; mkdir -p $O
RTX_LIB=$R/3360-ray-tracer_amd/variants/librtx_sc.so timeout -k 10 600 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_parity.py -m gpu -x -q -k "bunny or c3 or schedule" --timeout 300 --timeout-method thread > $O/pytest_sc.log 2>&1 || { tail -30 $O/pytest_sc.log; exit 1; }
tail -1 $O/pytest_sc.log
for r in 1 2; do
  for v in product sc; do
    lib="$R/3360-ray-tracer_amd/librtx.so"; [ $v = sc ] && lib="$R/3360-ray-tracer_amd/variants/librtx_sc.so"
    for a in "--workload c3_bunny" "--adaptive --workload c3_bunny"; do
      RTX_LIB=$lib timeout -k 10 200 python bench.py $a --schedule park --no-cpu-baseline --no-generic-leg --no-adaptive-leg > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', '$a', round(d['value'],1), round(d['ms_per_step'],3))"
    done
  done
done
