#!/bin/bash
# Re-verify the tree after the GEMM planner change: smoke, full GPU suite, flagship bench, the
# ResNet configs, a further planner A/B, kernel tables of the ResNet-20 and flagship steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
B="timeout -k 10 200 python -u benchmarks/run.py"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1 || exit 1
: > gpurun_out/v2_ab.txt
for cfg in "cifar_resnet" "cifar_resnet --depth 56" "resnet50 --batch 64" "resnet50 --batch 8"; do
  echo "default $cfg :: $($B $cfg --steps 20 --warmup 5 | tail -1 | cut -c60-140)" >> gpurun_out/v2_ab.txt || exit 1
  echo "t128min512 $cfg :: $(HOPSX_GEMM_T128_MIN=512 $B $cfg --steps 20 --warmup 5 | tail -1 | cut -c60-140)" >> gpurun_out/v2_ab.txt || exit 1
  echo "t64min512 $cfg :: $(HOPSX_GEMM_T64_MIN=512 $B $cfg --steps 20 --warmup 5 | tail -1 | cut -c60-140)" >> gpurun_out/v2_ab.txt || exit 1
done
echo "bn_coop_off cifar :: $(HOPSX_DISABLE=bn_coop $B cifar_resnet --steps 20 --warmup 5 | tail -1 | cut -c60-140)" >> gpurun_out/v2_ab.txt || exit 1
echo "bn_coop_off r50b64 :: $(HOPSX_DISABLE=bn_coop $B resnet50 --batch 64 --steps 20 --warmup 5 | tail -1 | cut -c60-140)" >> gpurun_out/v2_ab.txt || exit 1
echo "titanic :: $($B titanic --steps 200 --warmup 20 | tail -1 | cut -c1-160)" >> gpurun_out/v2_ab.txt || exit 1
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_cifar" -o run --output-format csv -- python3 "$R/benchmarks/run.py" cifar_resnet --steps 30 --warmup 10 > "$R/gpurun_out/prof_cifar.log" 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_flag" -o run --output-format csv -- python3 "$R/bench.py" --steps 100 --warmup 20 > "$R/gpurun_out/prof_flag.log" 2>&1
