#!/bin/bash
# first GPU pass: train tests, bench at a few batch sizes, rocprof of the flagship step
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m pytest tests/test_train_gpu.py -q -p no:cacheprovider > gpurun_out/train.log 2>&1
echo "EXIT train $?" >> gpurun_out/train.log
for B in 32 256 2048; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu $B --no-taxi > gpurun_out/bench_b$B.log 2>&1 || { echo "bench B=$B failed rc=$?" >> gpurun_out/bench_b$B.log; exit 1; }
done
timeout -k 10 200 python bench.py --steps 100 --warmup 20 --no-graph --no-taxi > gpurun_out/bench_nograph.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_b32" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 10 --no-taxi > "$GRAFT_REPO_ROOT/gpurun_out/prof_b32.log" 2>&1
echo "EXIT prof $?" >> "$GRAFT_REPO_ROOT/gpurun_out/prof_b32.log"
