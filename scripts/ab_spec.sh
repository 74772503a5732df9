#!/bin/bash
# A/B of speculative-walk variants (RTX_LEAF_SPEC) on C3: bit-compare, launch shape, rates
#   scripts/ab_spec.sh NAME lib1.so lib2.so ...   (NAME's library is the one bit-compared)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && V=3360-ray-tracer_amd/variants
S=${1:-spec}; shift
timeout -k 10 300 python scripts/cmp_libs.py 3360-ray-tracer_amd/librtx.so $V/librtx_$S.so > gpurun_out/cmp_${S}_bitexact.txt 2>&1 || exit $?
RTX_DEBUG_LAUNCH=1 RTX_LIB=$PWD/$V/librtx_$S.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-generic-leg --steps 3 --warmup 1 > gpurun_out/dbg_$S.json 2> gpurun_out/dbg_$S.err || exit $?
timeout -k 10 900 bash scripts/ab.sh ${S}_c3 "--no-generic-leg" default "$@"
