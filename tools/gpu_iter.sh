#!/bin/bash
# iteration pass: all GPU tests, flagship bench at reference batch and large batch, rocprof kernel stats
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${1:-it}
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/${TAG}_tests.log 2>&1
echo "EXIT tests $?" >> gpurun_out/${TAG}_tests.log
for B in 32 256 2048; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 30 --batch-per-gpu $B --no-taxi > gpurun_out/${TAG}_bench_b$B.log 2>&1 || { echo "bench B=$B failed rc=$?" >> gpurun_out/${TAG}_bench_b$B.log; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
for B in 32 2048; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_b$B" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 10 --no-taxi --batch-per-gpu $B > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_b$B.log" 2>&1 || exit 1
done
