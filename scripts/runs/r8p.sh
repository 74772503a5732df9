#!/bin/bash
# Round 5 (r8p): the fixed-spp accumulate with two chunks' loads in flight (previous build:
# variants/librtx_prev.so): GPU fixed-spp parity tests, C3 / C2 / C4 bench A/B (two interleaved
# rounds) and a kernel trace of the new build's accumulate bands.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8p; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for r in 1 2; do
  for v in prev acc2; do
    lib="$R/3360-ray-tracer_amd/librtx.so"; [ $v = prev ] && lib="$R/3360-ray-tracer_amd/variants/librtx_prev.so"
    for w in c3_bunny c2_final; do
      RTX_LIB=$lib timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-generic-leg --no-adaptive-leg > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v $w', round(d['value'],1), round(d['ms_per_step'],3), 'launch', round(d['roofline']['avg_launch_ms'],3))"
    done
  done
done
export TMPDIR=/tmp
cd /tmp || exit 1
for v in prev acc2; do
  lib="$R/3360-ray-tracer_amd/librtx.so"; [ $v = prev ] && lib="$R/3360-ray-tracer_amd/variants/librtx_prev.so"
  RTX_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/$O/trace_$v" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-generic-leg --no-adaptive-leg --schedule park --steps 20 > "$R/$O/trace_$v.json" 2> "$R/$O/trace_$v.err" || exit 1
done
echo traced
