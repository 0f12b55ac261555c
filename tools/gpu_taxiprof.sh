#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-tx}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/taxi_only.py" 50 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" 2>&1 || exit 1
python3 "$GRAFT_REPO_ROOT/tools/profsum.py" "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof/run_kernel_stats.csv" > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_profsum.txt"
