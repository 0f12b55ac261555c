#!/bin/bash
# Round 2: P2P failure handling + fused DP step on the one-GPU box (ranks share the device; gloo
# carries handle exchange / barriers / the reference all-reduce).  Then the bench's multi-rank path
# with the fused step inside the steps_per_execution graph, 2 and 4 ranks, and the fallback path.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_p2p_gpu.py tests/test_oneshot_gpu.py > gpurun_out/p2p_tests.log 2>&1 && \
HOPSX_DIST_BACKEND=gloo HOPSX_P2P=1 timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29651 tools/dp_fused_check.py > gpurun_out/dpfused4.log 2>&1 && \
HOPSX_DIST_BACKEND=gloo HOPSX_P2P=1 timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29652 bench.py --gpus 2 --steps 200 --warmup 20 > gpurun_out/bench_p2p2.log 2>&1 && \
HOPSX_DIST_BACKEND=gloo HOPSX_P2P=1 timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29653 bench.py --gpus 4 --steps 200 --warmup 20 > gpurun_out/bench_p2p4.log 2>&1 && \
HOPSX_DIST_BACKEND=gloo HOPSX_P2P=0 timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29654 bench.py --gpus 2 --steps 40 --warmup 10 --no-taxi > gpurun_out/bench_nop2p2.log 2>&1
rc=$?
echo "EXIT $rc" > gpurun_out/p2p_exit.txt
exit $rc
