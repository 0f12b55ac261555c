#!/bin/bash
# iteration pass: smoke, all GPU tests, flagship bench (default = driver config) + large batches, rocprof kernel stats
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${1:-it}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed rc=$?" >> gpurun_out/${TAG}_smoke.log; exit 1; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/${TAG}_tests.log 2>&1
echo "EXIT tests $?" >> gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench_default.log 2>&1 || { echo "bench default failed rc=$?" >> gpurun_out/${TAG}_bench_default.log; exit 1; }
for B in 256 2048; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 30 --batch-per-gpu $B --no-taxi > gpurun_out/${TAG}_bench_b$B.log 2>&1 || { echo "bench B=$B failed rc=$?" >> gpurun_out/${TAG}_bench_b$B.log; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_b32" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 10 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_b32.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_b2048" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 10 --no-taxi --batch-per-gpu 2048 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_b2048.log" 2>&1 || exit 1
