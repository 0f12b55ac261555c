#!/bin/bash
# Deferred BN finalize (apply kernels fold the replicas) + wgrad-MFMA K limit sweep: numerics tests,
# ResNet-20 / ResNet-50 A/B, kernel table of the ResNet-20 step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
B="timeout -k 10 200 python -u benchmarks/run.py"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_bnstats_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_kernels_v2_gpu.py \
  > gpurun_out/bn_tests.log 2>&1 && \
: > gpurun_out/ab.txt && \
echo "cifar default $($B cifar_resnet --steps 30 --warmup 10 | tail -1 | cut -c1-170)" >> gpurun_out/ab.txt && \
echo "cifar no_defer $(HOPSX_DISABLE=bn_defer $B cifar_resnet --steps 30 --warmup 10 | tail -1 | cut -c1-170)" >> gpurun_out/ab.txt && \
echo "cifar maxk640 $(HOPSX_WGRAD_MFMA_MAXK=640 $B cifar_resnet --steps 30 --warmup 10 | tail -1 | cut -c1-170)" >> gpurun_out/ab.txt && \
echo "r50 default $($B resnet50 --batch 64 --steps 20 --warmup 5 | tail -1 | cut -c1-170)" >> gpurun_out/ab.txt && \
echo "r50 no_defer $(HOPSX_DISABLE=bn_defer $B resnet50 --batch 64 --steps 20 --warmup 5 | tail -1 | cut -c1-170)" >> gpurun_out/ab.txt && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_cifar" -o run --output-format csv -- python3 "$R/benchmarks/run.py" cifar_resnet --steps 30 --warmup 10 > "$R/gpurun_out/prof_cifar.log" 2>&1
rc=$?
echo "EXIT $rc" >> "$R/gpurun_out/prof_cifar.log"
exit $rc
