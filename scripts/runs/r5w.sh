#!/bin/bash
# Round 4: adaptive early output with the copies issued from the host once the output is ready
# (no device-side wait on the copy stream): parity, interleaved A/B, a kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5w; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_timed.py \
  -k "render_multi or adaptive" > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  for arm in early late; do
    a=""; [ $arm = late ] && a="--no-early-output"
    timeout -k 10 200 python bench.py --adaptive --no-cpu-baseline --no-generic-leg $a > $O/c3a_${arm}_$rep.json 2> $O/c3a_${arm}_$rep.err || exit 1
    python3 scripts/sweep_summary.py "c3a $arm rep $rep" $O/c3a_${arm}_$rep.json | tee -a $O/ab.txt
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --adaptive --no-cpu-baseline --no-generic-leg --steps 20 --schedule park > $GRAFT_REPO_ROOT/$O/trace.json 2> $GRAFT_REPO_ROOT/$O/trace.err || exit 1
echo done
