#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/diag3.log; : > $out
run() { timeout -k 10 150 python tools/diag_div2.py "$@" >> $out 2>&1 || { echo "fail $*" >> $out; exit 1; }; }
run 32 1 400 0
run 32 1 400 1
run 32 0 400 0
HOPSX_DISABLE=direct_conv run 32 1 400 0
HOPSX_DISABLE=splitk run 32 1 400 0
HOPSX_DISABLE=pool8 run 32 1 400 0
HOPSX_DISABLE=direct_conv,pool8,splitk,loss_thread,rowreduce run 32 1 400 0
run 256 1 400 0
