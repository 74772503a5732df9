#!/bin/bash
# Round 4: the phases' batch margin growth (1 + step x (phase - 1)) with the shared chunks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6b; mkdir -p $O
for rep in 1 2; do
  for st in 0 0.125 default 0.5; do
    a=""; [ $st != default ] && a="--adapt-tune phase_mstep=$st"
    timeout -k 10 200 python bench.py --adaptive --no-cpu-baseline --no-generic-leg $a > $O/c3a_${st}_$rep.json 2> $O/c3a_${st}_$rep.err || exit 1
    python3 scripts/sweep_summary.py "phase_mstep=$st rep $rep" $O/c3a_${st}_$rep.json | tee -a $O/ab.txt
  done
done
