#!/bin/bash
# Register/scratch usage of the persistent-kernel instantiations for a set of -D flags
# (device-only compile, no GPU):  scripts/kres.sh [capi|park] [-DNAME=V ...]
R=/root/repo/3360-ray-tracer_amd
TU=${1:-capi}; shift
if [ "$TU" = park ]; then F=""; SRC=csrc/rtx_park.hip
else F="-mllvm -amdgpu-disable-clustered-low-occupancy-reschedule"; SRC=csrc/rtx_capi.hip; fi
OUT=$(mktemp /tmp/kres.XXXXXX.s)
cd $R && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I/root/repo/include \
  -Icsrc -Ihost/include $F "$@" --cuda-device-only -S $SRC -o $OUT 2>/dev/null || exit 1
echo "kernel<STACK,FAST,COUNT,SCATTER,PARK,TK,LAMB,NOTEX,NODOF>  scratch_B sgpr vgpr vgpr_spill"
grep -A12 "\.name:.*k_persistent" $OUT | grep -E "\.name|private_segment|sgpr_count|vgpr_count|vgpr_spill" |
  paste - - - - - | awk '{print $2, $4, $6, $8, $10}' | sed 's/_ZN4rtxd12k_persistentI//; s/EEEvNS_10RenderArgsEPy//'
echo "asm: $OUT"
