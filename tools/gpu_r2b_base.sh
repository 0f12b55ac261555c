#!/bin/bash
# Round-2 re-entry baseline on a fresh box: smoke, GPU tests, default bench, CIFAR ResNet-20 /
# ResNet-50 benchmarks and a rocprofv3 kernel table of the ResNet-20 step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1 && \
timeout -k 10 200 python -u benchmarks/run.py cifar_resnet --steps 30 --warmup 10 > gpurun_out/cifar20.log 2>&1 && \
timeout -k 10 200 python -u benchmarks/run.py resnet50 --batch 64 --steps 20 --warmup 5 > gpurun_out/r50.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_cifar" -o run --output-format csv -- python3 "$R/benchmarks/run.py" cifar_resnet --steps 30 --warmup 10 > "$R/gpurun_out/prof_cifar.log" 2>&1
rc=$?
echo "EXIT $rc" >> "$R/gpurun_out/prof_cifar.log"
exit $rc
