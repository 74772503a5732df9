#!/bin/bash
# Round 5 (r9i): the final build's C3 adaptive profile (kernel trace + PMC passes over every phase
# launch, scripts/profile.sh) for the adaptive roofline's source (refill at 12 idle lanes).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
timeout -k 10 600 bash scripts/profile.sh r9i_c3a --adaptive --workload c3_bunny --schedule park || exit 1
echo "c3a profiled"
