#!/bin/bash
# Round 5 (r9a): the fixed-spp kernel's slot chunk (kChunkPark 512) at 128 / 256 / 1024 (variants chN):
# r8z measured a ~1.9 ms fixed cost per fixed-spp launch (16 spp: 3.14 ms for 1.2 ms of segments).
# Parity subset on ch128, then C3 at 16 and 200 spp, two interleaved rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r9a; mkdir -p $O
RTX_LIB=$R/3360-ray-tracer_amd/variants/librtx_ch128.so timeout -k 10 600 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_parity.py -m gpu -x -q -k "bunny or c3 or schedule" --timeout 300 --timeout-method thread > $O/pytest_ch128.log 2>&1 || { tail -30 $O/pytest_ch128.log; exit 1; }
tail -1 $O/pytest_ch128.log
for r in 1 2; do
  for v in product ch128 ch256 ch1024; do
    lib="$R/3360-ray-tracer_amd/librtx.so"; [ $v != product ] && lib="$R/3360-ray-tracer_amd/variants/librtx_$v.so"
    for spp in 16 200; do
      RTX_LIB=$lib timeout -k 10 200 python bench.py --workload c3_bunny --spp $spp --schedule park --no-cpu-baseline --no-generic-leg --no-adaptive-leg > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', $spp, round(d['value'],1), round(d['ms_per_step'],3), 'launch', round(d['roofline']['avg_launch_ms'],3))"
    done
  done
done
