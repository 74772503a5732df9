#!/bin/bash
# Round 4: fixed-spp frames in row order (rows most expensive first in every slot region, so
# the launch drains on sky paths): parity, then interleaved A/B against image order.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5k; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_timed.py \
  -k "row_order or frame_parts or banded_output or timed_kernel_builds_match" > $O/pytest_rows.log 2>&1 || { tail -5 $O/pytest_rows.log; exit 1; }
tail -2 $O/pytest_rows.log
B="--no-cpu-baseline --no-generic-leg --no-adaptive-leg"
for rep in 1 2; do
  for wl in c3_bunny c2_final c5_mixed; do
    for ro in 0 1; do
      timeout -k 10 200 python bench.py $B --workload $wl --row-order $ro > $O/${wl}_ro${ro}_$rep.json 2> $O/${wl}_ro${ro}_$rep.err || exit 1
      python3 - "$wl ro=$ro rep=$rep" $O/${wl}_ro${ro}_$rep.json >> $O/rows.txt <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:>24} {d['value']:9.1f} Mrays/s {d['ms_per_step']:.3f} ms/step hot {d['roofline']['avg_launch_ms']:.3f} ms")
PY
    done
  done
done
cat $O/rows.txt
