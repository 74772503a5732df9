#!/bin/bash
# One GPU session: parity tests, then benches.  Stops at the first abnormal exit
# (fault / abort / timeout); ordinary test failures (pytest rc 1) do not stop the benches.
#   scripts/gpu_round.sh <tag> ["<bench args>" ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${1:-run}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
shift
for args in "$@"; do
  name=$(echo "$args" | tr ' -' '__')
  timeout -k 10 400 python bench.py $args > gpurun_out/bench_${TAG}${name}.json 2> gpurun_out/bench_${TAG}${name}.err || exit $?
done
