#!/bin/bash
# Round 6 (r10h): the walk's leaf rounds (speculative walk) timed inside the walk region
# (RTX_DEBUG_REGIONS counting builds): C3 fixed / adaptive, and the default bench line.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r10h; mkdir -p $O
B="--no-cpu-baseline --no-generic-leg --no-adaptive-leg --steps 3 --warmup 1"
RTX_DEBUG_REGIONS=1 timeout -k 10 300 python bench.py $B > $O/regions_c3_bunny.json 2> $O/regions_c3_bunny.err || { tail -20 $O/regions_c3_bunny.err; exit 1; }
echo "c3 fixed: $(grep 'rtx regions' $O/regions_c3_bunny.err | tail -1)"
RTX_DEBUG_REGIONS=1 timeout -k 10 300 python bench.py $B --adaptive > $O/regions_c3_bunny_adaptive.json 2> $O/regions_c3_bunny_adaptive.err || { tail -20 $O/regions_c3_bunny_adaptive.err; exit 1; }
echo "c3 adaptive: $(grep 'rtx regions' $O/regions_c3_bunny_adaptive.err | tail -1)"
RTX_DEBUG_REGIONS=1 timeout -k 10 300 python bench.py $B --workload c4_bunny4k --spp 64 > $O/regions_c4_bunny4k.json 2> $O/regions_c4_bunny4k.err || { tail -20 $O/regions_c4_bunny4k.err; exit 1; }
echo "c4 (64 spp): $(grep 'rtx regions' $O/regions_c4_bunny4k.err | tail -1)"
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); a=d['adaptive']; c=d['cpu_baseline']
print('default', round(d['value'],1), round(d['ms_per_step'],3), 'adaptive', round(a['value'],1), 'cpu ref', c['value'], c.get('runs'), 'x', c.get('gpu_over_reference'), c.get('gpu_over_reference_spread'))"
echo done
