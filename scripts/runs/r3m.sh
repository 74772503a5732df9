# round-3: guided chunk sizes (A/B against the previous build): C3, C3 adaptive, C2, C3 at 16 spp
cd $GRAFT_REPO_ROOT && \
timeout -k 10 600 bash scripts/ab.sh r3m_c3 "--no-generic-leg" default 3360-ray-tracer_amd/variants/librtx_base.so && \
timeout -k 10 600 bash scripts/ab.sh r3m_c3a "--no-generic-leg --adaptive" default 3360-ray-tracer_amd/variants/librtx_base.so && \
timeout -k 10 600 bash scripts/ab.sh r3m_c2 "--no-generic-leg --workload c2_final" default 3360-ray-tracer_amd/variants/librtx_base.so && \
timeout -k 10 600 bash scripts/ab.sh r3m_c3s16 "--no-generic-leg --spp 16" default 3360-ray-tracer_amd/variants/librtx_base.so
