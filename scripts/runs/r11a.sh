#!/bin/bash
# Round 6 (r11a): m: shading takes the winner's material from the walk and the primitive kind
# from the build (single-kind scenes: no dependent load of the record before the normal and the
# material); bwsl: barriers after the node and primitive loads + walk 1 / shade 0; bwslm: both;
# n1wslm: bwslm with the node-load barrier as priority 0 -> 1.  C3 fixed, interleaved.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
V=3360-ray-tracer_amd/variants
timeout -k 10 900 bash scripts/ab.sh r11a_c3 "--no-generic-leg --no-adaptive-leg" default $V/librtx_m.so $V/librtx_bwsl.so $V/librtx_bwslm.so $V/librtx_n1wslm.so || exit 1
echo done
