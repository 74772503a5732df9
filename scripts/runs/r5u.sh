#!/bin/bash
# Round 4: the phase floor (smallest phase while pixels remain) with the block-shared chunks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5u; mkdir -p $O
for rep in 1 2; do
  for ps in 2097152 4194304 default 16777216; do
    a=""; [ $ps != default ] && a="--adapt-tune phase_slots=$ps"
    timeout -k 10 200 python bench.py --adaptive --no-cpu-baseline --no-generic-leg $a > $O/c3a_${ps}_$rep.json 2> $O/c3a_${ps}_$rep.err || exit 1
    python3 scripts/sweep_summary.py "phase_slots=$ps rep $rep" $O/c3a_${ps}_$rep.json | tee -a $O/ab.txt
  done
done
