#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/diag5.log
timeout -k 10 300 python tools/diag_div4.py 12 300 32 graph >> $O 2>&1 || { echo "FAIL graph rc=$?" >> $O; exit 1; }
timeout -k 10 300 python tools/diag_div4.py 6 300 32 eager >> $O 2>&1 || { echo "FAIL eager rc=$?" >> $O; exit 1; }
HOPSX_DISABLE=direct_conv timeout -k 10 300 python tools/diag_div4.py 8 300 32 graph >> $O 2>&1 || { echo "FAIL nodirect rc=$?" >> $O; exit 1; }
HOPSX_DISABLE=splitk timeout -k 10 300 python tools/diag_div4.py 8 300 32 graph >> $O 2>&1 || { echo "FAIL nosplitk rc=$?" >> $O; exit 1; }
