#!/bin/bash
# Round 4: the default bench line, rocprofv3 kernel-trace + PMC passes of C3 (fixed and
# adaptive) and of the quantised-node variant (FETCH), and the 2-rank N>1 rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5l; mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
tail -1 $O/bench_default.json | cut -c1-300
timeout -k 10 900 bash scripts/profile.sh r5l_c3 || exit 1
echo "c3 profiled"
timeout -k 10 900 bash scripts/profile.sh r5l_c3a --adaptive || exit 1
echo "c3a profiled"
RTX_LIB=$PWD/3360-ray-tracer_amd/variants/librtx_qnode.so timeout -k 10 900 bash scripts/profile.sh r5l_c3_qnode || exit 1
echo "qnode profiled"
NPROC=2 timeout -k 10 450 bash scripts/multirank_rehearsal.sh || exit 1
cp gpurun_out/bench_rehearsal_2rank.json gpurun_out/bench_rehearsal_2rank.err $O/
tail -1 $O/bench_rehearsal_2rank.json | cut -c1-300
echo done
