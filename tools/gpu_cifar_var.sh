#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/cifar_var.txt
for D in "" "direct_conv"; do
  echo "DISABLE=$D $(HOPSX_DISABLE=$D timeout -k 5 200 python benchmarks/run.py cifar_resnet --steps 30 --warmup 10 2>/dev/null | tail -1 | cut -c1-160)" >> gpurun_out/cifar_var.txt || exit 1
done
echo "mnist $(timeout -k 5 200 python bench.py --no-taxi 2>/dev/null | tail -1 | cut -c150-260)" >> gpurun_out/cifar_var.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py tests/test_kernels_v2_gpu.py tests/test_models_gpu.py >> gpurun_out/cifar_var.txt 2>&1
