#!/bin/bash
# bench.py's N>1 path on a single GPU, exactly as an N-GPU run takes it (the default gloo group): NPROC ranks sharing
# cuda:0, rendering one C4 frame split in stripes into the shared /dev/shm framebuffer.
#   [NPROC=4] bash scripts/multirank_rehearsal.sh [bench args ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
N=${NPROC:-2}
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus $N --steps 2 --warmup 1 "$@" \
  > gpurun_out/bench_rehearsal_${N}rank.json 2> gpurun_out/bench_rehearsal_${N}rank.err
