#!/bin/bash
# Round 6 (r10u): pooled leaf rounds (variant librtx_pool: a leaf round tests all lanes' queued
# leaves at once, dealt out to every lane of the walk): GPU suite on the variant (parity), its
# launch shape, A/B against the product (C3, C3 adaptive, C4 at 256 spp); then the per-rank balance
# of 4-row stripes (C4, C5 at N = 2 / 4 / 8) and the 2-rank rehearsal with them.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r10u; mkdir -p $O
V=3360-ray-tracer_amd/variants
RTX_LIB=$R/$V/librtx_pool.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_pool.log 2>&1 || { tail -30 $O/pytest_gpu_pool.log; exit 1; }
tail -1 $O/pytest_gpu_pool.log
RTX_LIB=$R/$V/librtx_pool.so RTX_DEBUG_LAUNCH=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-generic-leg --no-adaptive-leg > $O/launch_pool.json 2> $O/launch_pool.err || { tail -5 $O/launch_pool.err; exit 1; }
grep "rtx launch" $O/launch_pool.err | sort | uniq -c | head -5
timeout -k 10 600 bash scripts/ab.sh r10u_c3 "--no-generic-leg --no-adaptive-leg" default $V/librtx_pool.so || exit 1
timeout -k 10 600 bash scripts/ab.sh r10u_c3a "--adaptive --no-generic-leg --no-adaptive-leg --steps 200" default $V/librtx_pool.so || exit 1
timeout -k 10 600 bash scripts/ab.sh r10u_c4 "--workload c4_bunny4k --spp 256 --no-generic-leg --no-adaptive-leg" default $V/librtx_pool.so || exit 1
cp gpurun_out/ab_r10u_*.txt $O/
timeout -k 10 400 python scripts/rank_balance.py --workload c4_bunny4k --ranks 2,4,8 --stripe-rows 4 > $O/rank_balance_c4_r4.jsonl 2> $O/rank_balance_c4_r4.err || { tail -20 $O/rank_balance_c4_r4.err; exit 1; }
timeout -k 10 400 python scripts/rank_balance.py --workload c5_mixed --ranks 2,4,8 --stripe-rows 4 --reps 1 > $O/rank_balance_c5_r4.jsonl 2> $O/rank_balance_c5_r4.err || { tail -20 $O/rank_balance_c5_r4.err; exit 1; }
python3 -c "
import json
for f in ('c4', 'c5'):
    for l in open('$O/rank_balance_'+f+'_r4.jsonl'):
        d=json.loads(l); print(d['workload'], d['stripe_rows'], d['n'], 'imb time %.4f seg %.4f pred %.0f one-gpu %.0f' % (d['imbalance_time'], d['imbalance_segments'], d['predicted_value_Mrays'], d['one_gpu_equiv_Mrays']))"
NPROC=2 timeout -k 10 500 bash scripts/multirank_rehearsal.sh --spp 32 || { tail -20 gpurun_out/bench_rehearsal_2rank.err; exit 1; }
cp gpurun_out/bench_rehearsal_2rank.json $O/
python3 -c "
import json; d=json.loads(open('$O/bench_rehearsal_2rank.json').read().strip().splitlines()[-1]); print('rehearsal', round(d['value'],1), 'rows covered', d['config']['frame_rows_covered'], d['config']['parallelism'])"
echo done
