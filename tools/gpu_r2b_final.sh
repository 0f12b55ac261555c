#!/bin/bash
# Round-2 end-of-session verification: smoke, full GPU suite, flagship bench, every ResNet config,
# kernel tables of the flagship / ResNet-20 / ResNet-50 steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
B="timeout -k 10 200 python -u benchmarks/run.py"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1 || exit 1
: > gpurun_out/final_bench.txt
for cfg in "cifar_resnet" "cifar_resnet --depth 56" "resnet50 --batch 64" "resnet50 --batch 8"; do
  echo "$cfg :: $($B $cfg --steps 30 --warmup 10 | tail -1 | cut -c1-190)" >> gpurun_out/final_bench.txt || exit 1
done
echo "titanic :: $($B titanic --steps 200 --warmup 20 | tail -1 | cut -c1-160)" >> gpurun_out/final_bench.txt || exit 1
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_cifar" -o run --output-format csv -- python3 "$R/benchmarks/run.py" cifar_resnet --steps 30 --warmup 10 > "$R/gpurun_out/prof_cifar.log" 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r50" -o run --output-format csv -- python3 "$R/benchmarks/run.py" resnet50 --batch 64 --steps 10 --warmup 5 > "$R/gpurun_out/prof_r50.log" 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_flag" -o run --output-format csv -- python3 "$R/bench.py" --steps 100 --warmup 20 > "$R/gpurun_out/prof_flag.log" 2>&1
