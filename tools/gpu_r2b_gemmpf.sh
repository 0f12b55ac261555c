#!/bin/bash
# GEMM depth-2 prefetch: kernel tests touching the GEMM, ResNet-20/50 + MNIST bench, R50 kernel table.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
B="timeout -k 10 200 python -u benchmarks/run.py"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 && \
: > gpurun_out/ab3.txt && \
echo "cifar20 $($B cifar_resnet --steps 30 --warmup 10 | tail -1 | cut -c1-170)" >> gpurun_out/ab3.txt && \
echo "r50b64 $($B resnet50 --batch 64 --steps 20 --warmup 5 | tail -1 | cut -c1-170)" >> gpurun_out/ab3.txt && \
echo "r50b8 $($B resnet50 --batch 8 --steps 20 --warmup 5 | tail -1 | cut -c1-170)" >> gpurun_out/ab3.txt && \
echo "mnist $(timeout -k 10 200 python -u bench.py | tail -1 | cut -c1-200)" >> gpurun_out/ab3.txt && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r50" -o run --output-format csv -- python3 "$R/benchmarks/run.py" resnet50 --batch 64 --steps 10 --warmup 5 > "$R/gpurun_out/prof_r50.log" 2>&1
