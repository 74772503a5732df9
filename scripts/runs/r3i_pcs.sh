# round-3: which PC sampling configurations this GPU offers, then one short host-trap sampling run of C3 (one frame)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3i && export TMPDIR=/tmp && \
timeout -k 10 120 rocprofv3 -L > gpurun_out/r3i/list_avail.txt 2>&1; \
grep -i -A30 "pc.sampl" gpurun_out/r3i/list_avail.txt > gpurun_out/r3i/pcs_configs.txt; \
cd /tmp && timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d $GRAFT_REPO_ROOT/gpurun_out/r3i/pcs -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-generic-leg --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r3i/bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/r3i/pcs.err
