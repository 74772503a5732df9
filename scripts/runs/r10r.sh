#!/bin/bash
# Round 6 (r10r): the generic (unspecialised) build under each schedule on the bunny: the PARK
# generic build spills 32 VGPRs, the plain one 3 (C3, C4 at 256 spp).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r10r; mkdir -p $O
for r in 1 2; do
  for sch in park plain; do
    timeout -k 10 300 python bench.py --generic --schedule $sch --no-cpu-baseline --no-generic-leg --no-adaptive-leg > $O/c3_${sch}_$r.json 2> $O/c3_${sch}_$r.err || { tail -5 $O/c3_${sch}_$r.err; exit 1; }
    timeout -k 10 300 python bench.py --generic --schedule $sch --workload c4_bunny4k --spp 256 --no-cpu-baseline --no-generic-leg --no-adaptive-leg > $O/c4_${sch}_$r.json 2> $O/c4_${sch}_$r.err || { tail -5 $O/c4_${sch}_$r.err; exit 1; }
  done
done
python3 -c "
import json,glob
for f in sorted(glob.glob('$O/*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f.split('/')[-1], round(d['value'],1), d['config']['kernel_build'])"
echo done
