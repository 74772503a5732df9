#!/bin/bash
# Round 4: fixed-spp frames in parts (the later parts' launches fill the earlier ones' drains,
# their accumulates run in the next part's drain): parity, then C3 A/B of part counts / shares.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5i; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_timed.py \
  -k "frame_parts or banded_output or render_multi" > $O/pytest_parts.log 2>&1 || exit 1
B="--no-cpu-baseline --no-generic-leg --no-adaptive-leg"
for fp in 1 2:0.25 default 2:0.15 3:0.15 4:0.1 2:0.4 1; do
  a=""; [ "$fp" != default ] && a="--frame-parts $fp"
  timeout -k 10 120 python bench.py $B $a > $O/c3_$fp.json 2> $O/c3_$fp.err || exit 1
  python3 - "$fp" $O/c3_$fp.json >> $O/parts.txt <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:>8} {d['value']:9.1f} Mrays/s {d['ms_per_step']:.3f} ms/step hot {d['roofline']['avg_launch_ms']:.3f} ms")
PY
done
cat $O/parts.txt
