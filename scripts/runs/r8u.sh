#!/bin/bash
# Round 5 (r8u): adaptive early output (the whole output copied to the pinned framebuffer while
# the last phases run, the remaining pixels patched in by the device): the new multi-device test
# first, then the GPU suite, then C3 / C2 adaptive against the previous build (variants/librtx_prev.so).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8u; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_timed.py -m gpu -x -v -k "early_output" --timeout 200 --timeout-method thread > $O/pytest_early.log 2>&1 || { tail -30 $O/pytest_early.log; exit 1; }
tail -2 $O/pytest_early.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for r in 1 2; do
  for v in prev early; do
    lib="$R/3360-ray-tracer_amd/librtx.so"; [ $v = prev ] && lib="$R/3360-ray-tracer_amd/variants/librtx_prev.so"
    for w in c3_bunny c2_final; do
      RTX_LIB=$lib timeout -k 10 200 python bench.py --adaptive --workload $w --no-cpu-baseline --no-generic-leg > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v $w', round(d['value'],1), round(d['ms_per_step'],3), d.get('rms_vs_cpu'), d.get('rms_check',{}).get('sample_counts_identical'))"
    done
  done
done
