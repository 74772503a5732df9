# round-3 diagnostic: per-wave start / exhausted / end times of fixed-spp C3 launches (variant with
# RTX_DIAG_WAVETIMES: fixed spp only), then the C5 CPU calibration case again (texture found by file name)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3l && \
for spp in 1 16 200; do RTX_LIB=$PWD/3360-ray-tracer_amd/variants/librtx_wt.so timeout -k 10 300 python bench.py --spp $spp --no-generic-leg --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r3l/c3_spp$spp.json 2> gpurun_out/r3l/c3_spp$spp.err || exit 1; done && \
timeout -k 10 600 python scripts/calibrate_cpu.py --threads 16 --only c5_mixed --out gpurun_out/r3l/cpu_calibration_16t_c5.json --host "GPU box host (MI355X pool), 16 threads" > gpurun_out/r3l/calibrate.out 2>&1
