# Rehearse the world_size>1 bench path (DP bucketed all-reduce between graph segments) with
# 2 ranks sharing the one GPU of a gpurun box.  gloo carries the collective (RCCL refuses two
# ranks per device); the 8-GPU RCCL run is the driver's.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
HOPSX_DIST_BACKEND=gloo timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 40 --warmup 10 \
  > gpurun_out/dist_gloo2.log 2>&1 && \
HOPSX_DIST_BACKEND=gloo timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 4 --steps 40 --warmup 10 \
  > gpurun_out/dist_gloo4.log 2>&1
