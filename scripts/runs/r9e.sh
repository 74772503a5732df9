#!/bin/bash
# Round 5 (r9e): the final build's profiles (non-temporal radiance records): C3 fixed and C3
# adaptive, kernel trace + PMC passes (scripts/profile.sh), for the rooflines' sources.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
timeout -k 10 600 bash scripts/profile.sh r9e_c3 --workload c3_bunny --schedule park || exit 1
echo "c3 profiled"
timeout -k 10 600 bash scripts/profile.sh r9e_c3a --adaptive --workload c3_bunny --schedule park || exit 1
echo "c3a profiled"
