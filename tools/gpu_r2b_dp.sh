#!/bin/bash
# Multi-rank rehearsal on the one-GPU box after the round-2 ResNet work: P2P tests, the flagship
# bench at 2 ranks (fused P2P DP step), CIFAR ResNet-20 collective all-reduce at 2 ranks (P2P fused
# step and the gloo fallback).  Ranks share the GPU: peer reads are local memory, not xGMI.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
L="timeout -k 10 240 python -u -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_p2p_gpu.py tests/test_oneshot_gpu.py > gpurun_out/p2p_tests.log 2>&1 && \
HOPSX_DIST_BACKEND=gloo HOPSX_P2P=1 $L --nproc-per-node 2 --master-port 29661 bench.py --gpus 2 --steps 200 --warmup 20 \
  > gpurun_out/bench_p2p2.log 2>&1 && \
HOPSX_DIST_BACKEND=gloo HOPSX_P2P=1 $L --nproc-per-node 2 --master-port 29662 benchmarks/run.py cifar_resnet --steps 30 --warmup 10 \
  > gpurun_out/cifar_p2p2.log 2>&1 && \
HOPSX_DIST_BACKEND=gloo HOPSX_P2P=0 $L --nproc-per-node 2 --master-port 29663 benchmarks/run.py cifar_resnet --steps 20 --warmup 5 \
  > gpurun_out/cifar_gloo2.log 2>&1
