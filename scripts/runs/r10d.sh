#!/bin/bash
# Round 6 (r10d): the chunk word + per-schedule shared chunk sizes (plain 256, PARK 128): GPU
# suite and the default bench line; then the available PC-sampling configurations and one short
# stochastic PC-sampling run of the C3 frame (the dynamic instruction mix by code region).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r10d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
timeout -k 10 400 python bench.py --no-cpu-baseline --workload c2_final > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
python3 -c "
import json
for w in ('c3','c2'):
    d=json.loads(open('$O/bench_'+w+'.json').read().strip().splitlines()[-1]); a=d['adaptive']; r=d['roofline']
    print(w, round(d['value'],1), round(d['ms_per_step'],3), 'adaptive', round(a['value'],1), round(a['ms_per_step'],3), 'frac', r.get('frac'), r.get('frac_class_priced'), 'l2', r['bytes_touched'].get('l2_frac'))"
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/rocprof_list.txt 2>&1 || echo "list rc $?"
grep -i -A12 "pc.sampl\|PC Sampling" $O/rocprof_list.txt | head -40
cd /tmp
timeout -k 10 -s KILL 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit instructions --pc-sampling-interval 1048576 -d "$R/$O/pcs" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-generic-leg --no-adaptive-leg --schedule park > "$R/$O/pcs_bench.json" 2> "$R/$O/pcs.err"; echo "pcs rc $?"
tail -5 "$R/$O/pcs.err"; ls -la "$R/$O/pcs" "$R/$O/pcs"/* 2>/dev/null | head
echo done
