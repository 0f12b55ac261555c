#!/bin/bash
# Residual gradient added in the conv-a dgrad epilogue: tests, ResNet A/B vs HOPSX_DISABLE=res_addend.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B="timeout -k 10 200 python -u benchmarks/run.py"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_bnstats_gpu.py tests/test_kernels_v2_gpu.py tests/test_models_gpu.py tests/test_graph_replay_gpu.py \
  > gpurun_out/ad_tests.log 2>&1 || exit 1
: > gpurun_out/ad.txt
for cfg in "cifar_resnet" "cifar_resnet --depth 56"; do
  echo "on $cfg :: $($B $cfg --steps 30 --warmup 10 | tail -1 | cut -c60-150)" >> gpurun_out/ad.txt || exit 1
  echo "off $cfg :: $(HOPSX_DISABLE=res_addend $B $cfg --steps 30 --warmup 10 | tail -1 | cut -c60-150)" >> gpurun_out/ad.txt || exit 1
  echo "on $cfg :: $($B $cfg --steps 30 --warmup 10 | tail -1 | cut -c60-150)" >> gpurun_out/ad.txt || exit 1
done
