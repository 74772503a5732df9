#!/bin/bash
# Round 6 (r10t): per-rank balance of 4-row stripes (the bench's new default) at N = 2 / 4 / 8 for
# C4 and C5, and the 2-rank rehearsal with them.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r10t; mkdir -p $O
timeout -k 10 400 python scripts/rank_balance.py --workload c4_bunny4k --ranks 2,4,8 --stripe-rows 4 > $O/rank_balance_c4_r4.jsonl 2> $O/rank_balance_c4_r4.err || { tail -20 $O/rank_balance_c4_r4.err; exit 1; }
timeout -k 10 400 python scripts/rank_balance.py --workload c5_mixed --ranks 2,4,8 --stripe-rows 4 --reps 1 > $O/rank_balance_c5_r4.jsonl 2> $O/rank_balance_c5_r4.err || { tail -20 $O/rank_balance_c5_r4.err; exit 1; }
python3 -c "
import json
for f in ('c4', 'c5'):
    for l in open('$O/rank_balance_'+f+'_r4.jsonl'):
        d=json.loads(l); print(d['workload'], d['stripe_rows'], d['n'], 'imb time %.4f seg %.4f pred %.0f one-gpu %.0f' % (d['imbalance_time'], d['imbalance_segments'], d['predicted_value_Mrays'], d['one_gpu_equiv_Mrays']))"
NPROC=2 timeout -k 10 500 bash scripts/multirank_rehearsal.sh --spp 32 || { tail -20 gpurun_out/bench_rehearsal_2rank.err; exit 1; }
cp gpurun_out/bench_rehearsal_2rank.json $O/
tail -1 $O/bench_rehearsal_2rank.json | cut -c1-200
python3 -c "
import json; d=json.loads(open('$O/bench_rehearsal_2rank.json').read().strip().splitlines()[-1]); print('rows covered', d['config']['frame_rows_covered'], d['config']['parallelism'])"
echo done
