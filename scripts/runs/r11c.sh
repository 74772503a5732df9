#!/bin/bash
# Round 6 (r11c): leaf rounds of the speculative walk at their own wave priority, on top of
# bwsl (barriers after the node and primitive loads, walk 1 / shading 0): lr2 above the node
# visits, lr0 below them.  C3 fixed and C3 adaptive, interleaved.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
V=3360-ray-tracer_amd/variants
timeout -k 10 900 bash scripts/ab.sh r11c_c3 "--no-generic-leg --no-adaptive-leg" default $V/librtx_bwsl.so $V/librtx_lr2.so $V/librtx_lr0.so || exit 1
timeout -k 10 900 bash scripts/ab.sh r11c_c3a "--adaptive --no-generic-leg --no-adaptive-leg" default $V/librtx_bwsl.so $V/librtx_lr2.so $V/librtx_lr0.so || exit 1
echo done
