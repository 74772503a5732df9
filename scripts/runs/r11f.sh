#!/bin/bash
# Round 6 (r11f): top: the speculative walk keeps its stack's top entry in a register, so a pop
# takes the next node without an LDS read on the path to the node's loads (the entry below is
# read then, for the next pop); q: the leaf queue's head entry in a register likewise; topq:
# both; topp: the top register in the plain walk (C2).  GPU suite on topq, then C3 fixed,
# C3 adaptive, C4, C2.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
V=3360-ray-tracer_amd/variants
O=gpurun_out/r11f; mkdir -p $O
RTX_LIB=$R/$V/librtx_topq.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_topq.log 2>&1 || { tail -30 $O/pytest_gpu_topq.log; exit 1; }
tail -1 $O/pytest_gpu_topq.log
N="--no-generic-leg --no-adaptive-leg"
timeout -k 10 900 bash scripts/ab.sh r11f_c3 "$N" default $V/librtx_top.so $V/librtx_q.so $V/librtx_topq.so || exit 1
timeout -k 10 900 bash scripts/ab.sh r11f_c3a "--adaptive $N" default $V/librtx_top.so $V/librtx_q.so $V/librtx_topq.so || exit 1
timeout -k 10 900 bash scripts/ab.sh r11f_c4 "--workload c4_bunny4k $N" default $V/librtx_top.so $V/librtx_q.so $V/librtx_topq.so || exit 1
timeout -k 10 900 bash scripts/ab.sh r11f_c2 "--workload c2_final $N" default $V/librtx_topp.so || exit 1
echo done
