#!/bin/bash
# Round 6 (r11g): the final build (load barriers, phase priority): GPU suite, smoke, and the rocprofv3 passes (kernel trace +
# PMC) of C3 fixed (PARK), C3 adaptive, C2 fixed and C2 adaptive for the bench's roofline.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r11g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 900 bash scripts/profile.sh r11g_c3 --schedule park || exit 1
timeout -k 10 900 bash scripts/profile.sh r11g_c3a --schedule park --adaptive || exit 1
timeout -k 10 900 bash scripts/profile.sh r11g_c2 --workload c2_final --schedule plain || exit 1
timeout -k 10 900 bash scripts/profile.sh r11g_c2a --workload c2_final --schedule plain --adaptive || exit 1
echo done
