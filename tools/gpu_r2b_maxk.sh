#!/bin/bash
# wgrad-MFMA K limit 640: kernel tests under it (pair KS=9 now reachable), ResNet-50 / ResNet-20 A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B="timeout -k 10 200 python -u benchmarks/run.py"
HOPSX_WGRAD_MFMA_MAXK=640 timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_v2_gpu.py tests/test_bnstats_gpu.py tests/test_models_gpu.py > gpurun_out/maxk_tests.log 2>&1 && \
: > gpurun_out/ab2.txt && \
echo "r50 maxk640 $(HOPSX_WGRAD_MFMA_MAXK=640 $B resnet50 --batch 64 --steps 20 --warmup 5 | tail -1 | cut -c1-170)" >> gpurun_out/ab2.txt && \
echo "r50 default $($B resnet50 --batch 64 --steps 20 --warmup 5 | tail -1 | cut -c1-170)" >> gpurun_out/ab2.txt && \
echo "r50b8 maxk640 $(HOPSX_WGRAD_MFMA_MAXK=640 $B resnet50 --batch 8 --steps 20 --warmup 5 | tail -1 | cut -c1-170)" >> gpurun_out/ab2.txt && \
echo "r50b8 default $($B resnet50 --batch 8 --steps 20 --warmup 5 | tail -1 | cut -c1-170)" >> gpurun_out/ab2.txt && \
echo "cifar56 maxk640 $(HOPSX_WGRAD_MFMA_MAXK=640 $B cifar_resnet --depth 56 --steps 30 --warmup 10 | tail -1 | cut -c1-170)" >> gpurun_out/ab2.txt && \
echo "cifar56 default $($B cifar_resnet --depth 56 --steps 30 --warmup 10 | tail -1 | cut -c1-170)" >> gpurun_out/ab2.txt
