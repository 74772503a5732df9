#!/bin/bash
# Round 6 (r10k): the generic (unspecialised) PARK builds with the restated small-argument cos/sin
# (the Lambertian-only builds keep the library's): A/B of the generic C3 frame (--generic), and
# the product's C3 line beside it (its ISA is unchanged).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r10k; mkdir -p $O
V=3360-ray-tracer_amd/variants
timeout -k 10 600 bash scripts/ab.sh r10k_generic "--generic --no-generic-leg --no-adaptive-leg" default $V/librtx_scgen.so || exit 1
timeout -k 10 600 bash scripts/ab.sh r10k_c5generic "--workload c5_mixed --generic --no-generic-leg --no-adaptive-leg --spp 256" default $V/librtx_scgen.so || exit 1
cp gpurun_out/ab_r10k_*.txt $O/
echo done
