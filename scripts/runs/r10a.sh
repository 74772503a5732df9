#!/bin/bash
# Round 6 (r10a): the adaptive phase kernel (MAP 1, block-shared chunks) over exactly the fixed-spp
# C3 frame's samples (adaptive with min_spp = spp = 200: one uniform first pass, nothing after it)
# against the fixed-spp kernel (MAP 0): interleaved timing, then a PMC profile of each.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r10a; mkdir -p $O
B="--no-cpu-baseline --no-generic-leg --no-adaptive-leg --schedule park"
for r in 1 2; do
  timeout -k 10 200 python bench.py $B > $O/map0_$r.json 2> $O/map0_$r.err || { tail -20 $O/map0_$r.err; exit 1; }
  timeout -k 10 200 python bench.py $B --adaptive --min-spp 200 > $O/map1u_$r.json 2> $O/map1u_$r.err || { tail -20 $O/map1u_$r.err; exit 1; }
  python3 -c "
import json
for t in ('map0_$r', 'map1u_$r'):
    d=json.loads(open('$O/'+t+'.json').read().strip().splitlines()[-1]); r=d['roofline']
    print(t, round(d['value'],1), round(d['ms_per_step'],3), 'launch ms', round(r['avg_launch_ms'],3), 'launches/step', d['steps'] and None, 'nodes/seg', round(r['nodes_per_segment'],3), 'simd', r['simd_efficiency_nodes'], r['simd_efficiency_prims'])"
done
timeout -k 10 900 bash scripts/profile.sh r10a_map0 --schedule park || exit 1
timeout -k 10 900 bash scripts/profile.sh r10a_map1u --schedule park --adaptive --min-spp 200 || exit 1

timeout -k 10 300 python -u -m pytest tests/test_gpu_timed.py -k "early_output or stripe" -x -q --timeout 200 --timeout-method thread > $O/pytest_early.log 2>&1 || { tail -30 $O/pytest_early.log; exit 1; }
tail -1 $O/pytest_early.log
timeout -k 10 300 python scripts/rank_balance.py --workload c4_bunny4k --ranks 2,4,8 --stripe-rows 8 > $O/rank_balance_c4.jsonl 2> $O/rank_balance_c4.err || { tail -20 $O/rank_balance_c4.err; exit 1; }
python3 -c "
import json
for l in open('$O/rank_balance_c4.jsonl'):
    d=json.loads(l); print(d['workload'], d['stripe_rows'], d['n'], 'imb time %.4f seg %.4f pred %.0f one-gpu %.0f' % (d['imbalance_time'], d['imbalance_segments'], d['predicted_value_Mrays'], d['one_gpu_equiv_Mrays']))"
echo done
