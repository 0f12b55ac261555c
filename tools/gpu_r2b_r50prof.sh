#!/bin/bash
# Full GPU suite on the current tree + ResNet-50 B=64 and ResNet-20 kernel tables.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -u benchmarks/run.py cifar_resnet --steps 30 --warmup 10 > gpurun_out/cifar20.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r50" -o run --output-format csv -- python3 "$R/benchmarks/run.py" resnet50 --batch 64 --steps 10 --warmup 5 > "$R/gpurun_out/prof_r50.log" 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_cifar" -o run --output-format csv -- python3 "$R/benchmarks/run.py" cifar_resnet --steps 30 --warmup 10 > "$R/gpurun_out/prof_cifar.log" 2>&1
rc=$?
echo "EXIT $rc" >> "$R/gpurun_out/prof_r50.log"
exit $rc
