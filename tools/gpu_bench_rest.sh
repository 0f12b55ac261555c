#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${1:-it}
B=gpurun_out/${TAG}_benchmarks.log
for c in "cifar_resnet --steps 50 --warmup 10" "cifar_resnet --depth 56 --steps 30 --warmup 5" "resnet50 --steps 20 --warmup 5" "resnet50 --batch 64 --steps 20 --warmup 5" "mnist_mirrored --batch 2048 --steps 100 --warmup 10"; do
  echo "== $c" >> $B
  timeout -k 10 300 python benchmarks/run.py $c >> $B 2>&1 || { echo "FAIL rc=$? $c" >> $B; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_r50" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/benchmarks/run.py" resnet50 --batch 64 --steps 10 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_r50.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_b32" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 10 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_b32.log" 2>&1 || exit 1
