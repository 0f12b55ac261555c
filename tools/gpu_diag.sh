#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/diag4.log
run() { timeout -k 10 120 python tools/diag_div3.py "$@" >> $O 2>&1 || { echo "FAIL $* rc=$?" >> $O; exit 1; }; }
run 32 1 0 0 220
run 32 1 0 1 220
run 32 1 1 0 220
run 32 0 0 0 220
run 256 1 0 0 330
run 256 0 0 0 330
timeout -k 10 120 python bench.py --no-taxi >> $O 2>&1
HOPSX_GRAPH=0 timeout -k 10 120 python bench.py --no-taxi >> $O 2>&1
