# round-3 experiment: adaptive on one launch (variants from branch wip-adaptive-queue): phases (default) vs the
# ticket queue (q2) vs non-blocking claims on one ring with backed-off idle waves (q5); C3 adaptive, then C2
cd $GRAFT_REPO_ROOT && \
timeout -k 10 900 bash scripts/ab.sh r3s_c3a "--no-generic-leg --adaptive" default 3360-ray-tracer_amd/variants/librtx_q2.so 3360-ray-tracer_amd/variants/librtx_q5.so
