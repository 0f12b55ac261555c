# one-/two-shot all-reduce on the one-GPU box: 2 and 4 ranks sharing the device (bitwise checks,
# hipGraph replay, timing), then the bench's DP path with the kernel captured in the
# steps_per_execution graph (4 ranks: the MNIST bucket takes the two-shot path)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
HOPSX_DIST_BACKEND=gloo timeout -k 10 150 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29621 tools/oneshot_check.py > gpurun_out/oneshot2.log 2>&1 && \
HOPSX_DIST_BACKEND=gloo timeout -k 10 150 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29624 tools/oneshot_check.py > gpurun_out/oneshot4.log 2>&1 && \
HOPSX_DIST_BACKEND=gloo HOPSX_ONESHOT_AR=1 timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29623 bench.py --gpus 4 --steps 80 --warmup 10 \
  > gpurun_out/bench_oneshot4.log 2>&1
