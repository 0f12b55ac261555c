#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/perf1.log
timeout -k 10 300 python tools/gemm_bench.py >> $O 2>&1 || { echo "FAIL gemm rc=$?" >> $O; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/mb32" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/microbench.py" 32 200 >> "$GRAFT_REPO_ROOT/$O" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/mb2048" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/microbench.py" 2048 50 >> "$GRAFT_REPO_ROOT/$O" 2>&1 || exit 1
