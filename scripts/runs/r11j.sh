#!/bin/bash
# Round 6 (r11j): the final build (load barriers, phase priority) in one call: bench lines of
# the default (C3 + adaptive leg + the reference timed) and C2; rocprofv3 passes of C4 and C5,
# summarised on the box so their bench lines price the new profiles; C4 and C5 bench lines;
# the 2-rank rehearsal of the N > 1 path on one GPU (C4, 32 spp).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r11j; mkdir -p $O
line() {
  w=$1; A=""; [ $w != default ] && A="--workload $w"
  timeout -k 10 500 python bench.py $A > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; return 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_$w.json').read().strip().splitlines()[-1]); a=d.get('adaptive') or {}; c=d['cpu_baseline']; r=d['roofline']; g=d.get('generic_build') or {}
print('$w', round(d['value'],1), round(d['ms_per_step'],3), 'adaptive', round(a.get('value',0),1), 'generic', round(g.get('value',0),1), 'cpu', round(c['value'],3), c.get('kind'), 'x', round(c.get('gpu_over_reference',0),1), 'frac', round(r.get('frac') or 0,3), round(r.get('frac_class_priced') or 0,3), 'rms', d.get('rms_vs_cpu'))"
}
line default && line c2_final || exit 1
timeout -k 10 900 bash scripts/profile.sh r11h_c4 --workload c4_bunny4k --schedule park || exit 1
timeout -k 10 900 bash scripts/profile.sh r11h_c5 --workload c5_mixed --schedule plain || exit 1
python3 scripts/summarize_prof.py gpurun_out/prof_r11h_c4 r06 c4_bunny4k persistent fast > /dev/null || exit 1
python3 scripts/summarize_prof.py gpurun_out/prof_r11h_c5 r06 c5_mixed persistent fast > /dev/null || exit 1
line c4_bunny4k && line c5_mixed || exit 1
NPROC=2 timeout -k 10 500 bash scripts/multirank_rehearsal.sh --spp 32 || { tail -20 gpurun_out/bench_rehearsal_2rank.err; exit 1; }
cp gpurun_out/bench_rehearsal_2rank.json $O/
tail -1 $O/bench_rehearsal_2rank.json | cut -c1-400
echo done
