# round-3: the bunny's Lambertian texture-free builds reading only the camera from the kernel argument
# segment at refill (spilled SGPRs 79 -> 68) against the default (arguments in registers): C3, C3 adaptive
cd $GRAFT_REPO_ROOT && \
timeout -k 10 600 bash scripts/ab.sh r4n_c3 "--no-generic-leg" default 3360-ray-tracer_amd/variants/librtx_camkarg.so && \
timeout -k 10 600 bash scripts/ab.sh r4n_c3a "--no-generic-leg --adaptive" default 3360-ray-tracer_amd/variants/librtx_camkarg.so
