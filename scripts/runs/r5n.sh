#!/bin/bash
# Round 4: adaptive frames' early output copy (whole output during the last phases, patch list
# after): parity, then the adaptive bench line twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5n; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_timed.py \
  -k "render_multi or adaptive" > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
  timeout -k 10 200 python bench.py --adaptive --no-cpu-baseline --no-generic-leg > $O/c3a_$rep.json 2> $O/c3a_$rep.err || exit 1
  python3 scripts/sweep_summary.py "c3a rep $rep" $O/c3a_$rep.json
done
