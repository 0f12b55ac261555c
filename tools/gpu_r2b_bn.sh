#!/bin/bash
# BN statistics in the conv epilogue: numerics tests, ResNet-20 / ResNet-50 benchmarks (fused vs
# HOPSX_DISABLE=bnstats), kernel table of the ResNet-20 step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_bnstats_gpu.py "tests/test_kernels_gpu.py::test_batchnorm" tests/test_models_gpu.py > gpurun_out/bn_tests.log 2>&1 && \
timeout -k 10 200 python -u benchmarks/run.py cifar_resnet --steps 30 --warmup 10 > gpurun_out/cifar20.log 2>&1 && \
HOPSX_DISABLE=bnstats timeout -k 10 200 python -u benchmarks/run.py cifar_resnet --steps 30 --warmup 10 > gpurun_out/cifar20_nobns.log 2>&1 && \
timeout -k 10 200 python -u benchmarks/run.py resnet50 --batch 64 --steps 20 --warmup 5 > gpurun_out/r50.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_cifar" -o run --output-format csv -- python3 "$R/benchmarks/run.py" cifar_resnet --steps 30 --warmup 10 > "$R/gpurun_out/prof_cifar.log" 2>&1
rc=$?
echo "EXIT $rc" >> "$R/gpurun_out/prof_cifar.log"
exit $rc
