#!/bin/bash
# GEMM-dgrad + MFMA-wgrad paired launch: tests, ResNet A/B against HOPSX_DISABLE=bwd_pair_gemm.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B="timeout -k 10 200 python -u benchmarks/run.py"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_v2_gpu.py tests/test_bnstats_gpu.py tests/test_models_gpu.py tests/test_kernels_gpu.py \
  > gpurun_out/pg_tests.log 2>&1 || exit 1
: > gpurun_out/pg.txt
for cfg in "cifar_resnet" "cifar_resnet --depth 56" "resnet50 --batch 64" "resnet50 --batch 8"; do
  echo "on $cfg :: $($B $cfg --steps 30 --warmup 10 | tail -1 | cut -c60-150)" >> gpurun_out/pg.txt || exit 1
  echo "off $cfg :: $(HOPSX_DISABLE=bwd_pair_gemm $B $cfg --steps 30 --warmup 10 | tail -1 | cut -c60-150)" >> gpurun_out/pg.txt || exit 1
done
