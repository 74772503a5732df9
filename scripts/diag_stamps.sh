#!/bin/bash
# Diagnostic builds on a few workloads: region cycle split (RTX_STAMPS) and the node-loop
# active-lane histogram (RTX_TAILHIST, counting pass).  Output: gpurun_out/diag_*.txt
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" || exit 1
mkdir -p gpurun_out
for w in "c3_bunny --schedule park" "c3_bunny --schedule plain" "c2_final --schedule plain" "c5_mixed --spp 16 --schedule plain"; do
  n=$(echo $w | tr ' -' '__')
  RTX_LIB=$R/3360-ray-tracer_amd/variants/librtx_stamps.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-generic-leg --steps 3 --warmup 1 --workload $w > gpurun_out/diag_stamps_$n.json 2> gpurun_out/diag_stamps_$n.txt || exit $?
  RTX_LIB=$R/3360-ray-tracer_amd/variants/librtx_tail.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-generic-leg --steps 1 --warmup 1 --workload $w > gpurun_out/diag_tail_$n.json 2> gpurun_out/diag_tail_$n.txt || exit $?
done
