# round-3: statistics counters read back with the frame (pinned async copy before the end event) instead of a
# blocking copy after it: GPU tests + smoke, A/B of the step time against the previous library on C3 and C2
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4k && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r4k/pytest.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4k/smoke.log 2>&1 && \
timeout -k 10 600 bash scripts/ab.sh r4k_c3 "--no-generic-leg" default 3360-ray-tracer_amd/variants/librtx_head.so && \
timeout -k 10 600 bash scripts/ab.sh r4k_c2 "--no-generic-leg --workload c2_final" default 3360-ray-tracer_amd/variants/librtx_head.so
