#!/bin/bash
# XCD-aware dgrad block order (HOPSX_DGRAD_XCD=1): tests under it, then A/B on ResNet-20/56 and MNIST.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B="timeout -k 10 200 python -u benchmarks/run.py"
HOPSX_DGRAD_XCD=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_v2_gpu.py tests/test_bnstats_gpu.py tests/test_models_gpu.py tests/test_graph_replay_gpu.py \
  > gpurun_out/xcd_tests.log 2>&1 || exit 1
: > gpurun_out/xcd.txt
for cfg in "cifar_resnet" "cifar_resnet --depth 56"; do
  for r in 1 2; do
    echo "off $cfg :: $($B $cfg --steps 30 --warmup 10 | tail -1 | cut -c60-140)" >> gpurun_out/xcd.txt || exit 1
    echo "on $cfg :: $(HOPSX_DGRAD_XCD=1 $B $cfg --steps 30 --warmup 10 | tail -1 | cut -c60-140)" >> gpurun_out/xcd.txt || exit 1
  done
done
echo "off mnist :: $(timeout -k 10 200 python -u bench.py --no-taxi | tail -1 | cut -c60-200)" >> gpurun_out/xcd.txt || exit 1
echo "on mnist :: $(HOPSX_DGRAD_XCD=1 timeout -k 10 200 python -u bench.py --no-taxi | tail -1 | cut -c60-200)" >> gpurun_out/xcd.txt || exit 1
