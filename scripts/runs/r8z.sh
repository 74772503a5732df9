#!/bin/bash
# Round 5 (r8z): launch time of the fixed-spp C3 kernel against its spp (16 / 32 / 64 / 200), with the
# counting pass's timeline (RTX_DEBUG_DRAIN): the fixed cost of one launch, to set beside the adaptive
# frame's first phase (16 spp on the phase kernel, 2.38 ms in adaptive_frame_r8v_final.txt).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r8z; mkdir -p $O
for spp in 16 32 64 200; do
  RTX_DEBUG_DRAIN=1 timeout -k 10 200 python bench.py --workload c3_bunny --spp $spp --schedule park --no-cpu-baseline --no-generic-leg --no-adaptive-leg > $O/b$spp.json 2> $O/b$spp.err || { tail -20 $O/b$spp.err; exit 1; }
  grep -h "timeline" $O/b$spp.err | tail -2
  python3 -c "
import json; d=json.loads(open('$O/b$spp.json').read().strip().splitlines()[-1]); r=d['roofline']; print($spp, round(d['value'],1), round(d['ms_per_step'],3), 'launch', round(r['avg_launch_ms'],3), 'segs', r['segments_per_launch'])"
done
