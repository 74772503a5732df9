# round-3 diagnostic: launch timeline (10.24 us buckets: wave iterations, active lanes per iteration, wave exits) of
# fixed-spp C3 at 16 and 200 spp (diagnostic variant library), then the product's launch time against spp
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3h && \
RTX_LIB=$PWD/3360-ray-tracer_amd/variants/librtx_diag.so timeout -k 10 300 python bench.py --spp 16 --no-generic-leg --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3h/c3_spp16.json 2> gpurun_out/r3h/c3_spp16.err && \
RTX_LIB=$PWD/3360-ray-tracer_amd/variants/librtx_diag.so timeout -k 10 300 python bench.py --no-generic-leg --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r3h/c3_spp200.json 2> gpurun_out/r3h/c3_spp200.err && \
for spp in 1 2 4 8 16 32 64 128 200; do timeout -k 10 300 python bench.py --spp $spp --no-generic-leg --no-cpu-baseline > gpurun_out/r3h/sweep_$spp.json 2>> gpurun_out/r3h/sweep.err || exit 1; done
