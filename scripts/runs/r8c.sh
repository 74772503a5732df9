#!/bin/bash
# Round 5 (r8c): bench lines of C2 / C4 / C5 on the round-5 build (reference cpu_baseline), then
# stochastic PC sampling of the fixed-spp C3 frame (where the hot kernel's cycles go).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8c; mkdir -p $O
for w in c2_final c4_bunny4k c5_mixed; do
  timeout -k 10 400 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_$w.json').read().strip().splitlines()[-1]); print('$w', round(d['value'],1), round(d['ms_per_step'],3), d['roofline'].get('frac'), d['cpu_baseline']['value'])"
done
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
  --pc-sampling-interval 1048576 -d "$R/$O/pcs" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-generic-leg --no-adaptive-leg --schedule park --steps 3 --warmup 1 \
  > "$R/$O/pcs_bench.json" 2> "$R/$O/pcs.err"
rc=$?
echo "pc sampling rc=$rc"; tail -5 "$R/$O/pcs.err"
ls -la "$R/$O/pcs" 2>/dev/null | head
exit 0
