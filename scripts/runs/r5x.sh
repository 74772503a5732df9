#!/bin/bash
# Round 4: host-side timestamps of bench frames (RTX_DEBUG_HOST), fixed and adaptive; the
# adaptive output copy enqueued before the frame's end event; parity of the output paths.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5x; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_timed.py \
  -k "render_multi or banded" > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
RTX_DEBUG_HOST=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-generic-leg --no-adaptive-leg --steps 20 > $O/c3.json 2> $O/c3.err || exit 1
grep "rtx host" $O/c3.err | tail -5
RTX_DEBUG_HOST=1 timeout -k 10 200 python bench.py --adaptive --no-cpu-baseline --no-generic-leg --steps 20 > $O/c3a.json 2> $O/c3a.err || exit 1
grep "rtx host" $O/c3a.err | tail -5
for rep in 1 2; do
  timeout -k 10 200 python bench.py --adaptive --no-cpu-baseline --no-generic-leg > $O/c3a_$rep.json 2> $O/c3a_$rep.err || exit 1
  python3 scripts/sweep_summary.py "c3a rep $rep" $O/c3a_$rep.json
done
