#!/bin/bash
# Round 6 (r11i): the final build's bench lines (load barriers, phase priority): the default (C3 + its adaptive leg, the
# reference timed as CPU baseline), C2, C4 and C5 (each with its generic and adaptive legs).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r11i; mkdir -p $O
for w in default c2_final c4_bunny4k c5_mixed; do
  A=""; [ $w != default ] && A="--workload $w"
  timeout -k 10 500 python bench.py $A > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_$w.json').read().strip().splitlines()[-1]); a=d.get('adaptive') or {}; c=d['cpu_baseline']; r=d['roofline']; g=d.get('generic_build') or {}
print('$w', round(d['value'],1), round(d['ms_per_step'],3), 'adaptive', round(a.get('value',0),1), 'generic', round(g.get('value',0),1), 'cpu', round(c['value'],3), c.get('kind'), 'x', round(c.get('gpu_over_reference',0),1), 'frac', round(r.get('frac') or 0,3), round(r.get('frac_class_priced') or 0,3), 'rms', d.get('rms_vs_cpu'))"
done
echo done
