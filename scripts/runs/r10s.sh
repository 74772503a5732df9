#!/bin/bash
# Round 6 (r10s): the N > 1 bench path with 4 ranks sharing one GPU (C4, 32 spp) on the final
# build, and the per-rank balance of other stripe heights (4 / 16 rows) for C4 at N = 8.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r10s; mkdir -p $O
NPROC=4 timeout -k 10 500 bash scripts/multirank_rehearsal.sh --spp 32 || { tail -20 gpurun_out/bench_rehearsal_4rank.err; exit 1; }
cp gpurun_out/bench_rehearsal_4rank.json $O/
tail -1 $O/bench_rehearsal_4rank.json | cut -c1-300
timeout -k 10 400 python scripts/rank_balance.py --workload c4_bunny4k --ranks 8 --stripe-rows 4,16 > $O/rank_balance_c4_rows.jsonl 2> $O/rank_balance_c4_rows.err || { tail -20 $O/rank_balance_c4_rows.err; exit 1; }
python3 -c "
import json
for l in open('$O/rank_balance_c4_rows.jsonl'):
    d=json.loads(l); print(d['workload'], d['stripe_rows'], d['n'], 'imb time %.4f seg %.4f pred %.0f' % (d['imbalance_time'], d['imbalance_segments'], d['predicted_value_Mrays']))"
echo done
