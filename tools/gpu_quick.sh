#!/bin/bash
# quick pass: targeted GPU tests + flagship bench + per-op microbench under rocprof
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${1:-q}
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
echo "EXIT tests $?" >> gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed rc=$?" >> gpurun_out/${TAG}_bench.log; exit 1; }
timeout -k 10 300 python bench.py --batch-per-gpu 2048 --no-taxi --steps 100 >> gpurun_out/${TAG}_bench.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_mb32" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/microbench.py" 32 200 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_mb.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_b32" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 10 --no-taxi > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof_b32.log" 2>&1 || exit 1
