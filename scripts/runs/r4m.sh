# round-3: accumulate staging (k_accumulate_sum) 8 samples x 16 pixels (default) vs 16 x 16 vs 32 x 8 per
# workgroup, on C3 and C2 (the step time holds the accumulate's 8 bands)
cd $GRAFT_REPO_ROOT && \
timeout -k 10 600 bash scripts/ab.sh r4m_c3 "--no-generic-leg" default 3360-ray-tracer_amd/variants/librtx_acc_c16_p16.so 3360-ray-tracer_amd/variants/librtx_acc_c32_p8.so && \
timeout -k 10 600 bash scripts/ab.sh r4m_c2 "--no-generic-leg --workload c2_final" default 3360-ray-tracer_amd/variants/librtx_acc_c16_p16.so 3360-ray-tracer_amd/variants/librtx_acc_c32_p8.so && \
export TMPDIR=/tmp && cd /tmp && for v in acc_c16_p16 acc_c32_p8; do RTX_LIB=$GRAFT_REPO_ROOT/3360-ray-tracer_amd/variants/librtx_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4m_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-generic-leg --steps 20 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r4m_$v.json 2>/dev/null || exit $?; done
