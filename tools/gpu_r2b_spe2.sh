#!/bin/bash
# bench.py with 32 steps per graph: 1 rank at the driver's K/W, 2 ranks sharing the GPU (fused P2P step).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b1.log 2>&1 && \
HOPSX_DIST_BACKEND=gloo HOPSX_P2P=1 timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29671 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/b2.log 2>&1
