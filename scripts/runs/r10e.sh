#!/bin/bash
# Round 6 (r10e): where a persistent wave's time goes, by region of its loop (refill / walk /
# shading), from the counting builds' s_memtime stamps (RTX_DEBUG_REGIONS), for the bench's
# workloads; the GPU suite on the instrumented counting build first.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/r10e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
B="--no-cpu-baseline --no-generic-leg --no-adaptive-leg --steps 3 --warmup 1"
for w in c3_bunny c2_final c5_mixed; do
  RTX_DEBUG_REGIONS=1 timeout -k 10 300 python bench.py $B --workload $w > $O/regions_$w.json 2> $O/regions_$w.err || { tail -20 $O/regions_$w.err; exit 1; }
  echo "$w fixed: $(grep 'rtx regions' $O/regions_$w.err | tail -1)"
done
for w in c3_bunny c2_final; do
  RTX_DEBUG_REGIONS=1 timeout -k 10 300 python bench.py $B --workload $w --adaptive > $O/regions_${w}_adaptive.json 2> $O/regions_${w}_adaptive.err || { tail -20 $O/regions_${w}_adaptive.err; exit 1; }
  echo "$w adaptive: $(grep 'rtx regions' $O/regions_${w}_adaptive.err | tail -1)"
done
RTX_DEBUG_REGIONS=1 timeout -k 10 300 python bench.py $B --adaptive --min-spp 200 --schedule park > $O/regions_c3_map1u.json 2> $O/regions_c3_map1u.err || { tail -20 $O/regions_c3_map1u.err; exit 1; }
echo "c3 phase kernel on the fixed samples: $(grep 'rtx regions' $O/regions_c3_map1u.err | tail -1)"
echo done
