#!/bin/bash
# Round 6 (r10b): does the adaptive early output fire on the bench's path; A/B of the adaptive phase
# kernel's overhead (MAP 1: kernel arguments re-read at refill, per-wave chunks instead of the
# block-shared ones, both) on C3 adaptive and on the fixed frame's samples (min_spp = spp); per-rank
# load of the N-GPU split measured on one GPU (C4, C5).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r10b; mkdir -p $O
timeout -k 10 120 python scripts/diag_early_output.py > $O/diag_early_output.txt 2>&1 || { tail -20 $O/diag_early_output.txt; exit 1; }
cat $O/diag_early_output.txt
L="default 3360-ray-tracer_amd/variants/librtx_m1args.so 3360-ray-tracer_amd/variants/librtx_m1noshared.so 3360-ray-tracer_amd/variants/librtx_m1both.so"
timeout -k 10 600 bash scripts/ab.sh r10b_c3a "--adaptive --no-generic-leg --no-adaptive-leg --steps 200" $L || exit 1
timeout -k 10 600 bash scripts/ab.sh r10b_map1u "--adaptive --min-spp 200 --no-generic-leg --no-adaptive-leg --schedule park" $L || exit 1
cp gpurun_out/ab_r10b_*.txt $O/
timeout -k 10 300 python scripts/rank_balance.py --workload c4_bunny4k --ranks 2,4,8 --stripe-rows 8 > $O/rank_balance_c4.jsonl 2> $O/rank_balance_c4.err || { tail -20 $O/rank_balance_c4.err; exit 1; }
timeout -k 10 300 python scripts/rank_balance.py --workload c5_mixed --ranks 2,4,8 --stripe-rows 8 --reps 1 > $O/rank_balance_c5.jsonl 2> $O/rank_balance_c5.err || { tail -20 $O/rank_balance_c5.err; exit 1; }
python3 -c "
import json
for f in ('c4', 'c5'):
    for l in open('$O/rank_balance_'+f+'.jsonl'):
        d=json.loads(l); print(d['workload'], d['stripe_rows'], d['n'], 'imb time %.4f seg %.4f pred %.0f one-gpu %.0f' % (d['imbalance_time'], d['imbalance_segments'], d['predicted_value_Mrays'], d['one_gpu_equiv_Mrays']))"
echo done
