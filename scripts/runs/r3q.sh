# round-3: PARK-kernel choices re-checked with the speculative walk: restated small-argument cos/sin, the
# triangle test with early exits, park at 12 walking lanes, refill at 20 idle lanes (C3, A/B)
cd $GRAFT_REPO_ROOT && \
timeout -k 10 1000 bash scripts/ab.sh r3q_c3 "--no-generic-leg" default 3360-ray-tracer_amd/variants/librtx_sc1.so 3360-ray-tracer_amd/variants/librtx_tbr0.so 3360-ray-tracer_amd/variants/librtx_park12.so 3360-ray-tracer_amd/variants/librtx_refill20.so
