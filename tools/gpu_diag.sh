#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/diag.log; : > $out
for D in "" "direct_conv" "pool8" "rowreduce" "loss_thread" "splitk" "direct_conv,pool8,rowreduce,loss_thread,splitk"; do
  HOPSX_DISABLE="$D" timeout -k 10 120 python tools/diag_div.py 256 1 >> $out 2>&1 || { echo "fail $D" >> $out; exit 1; }
done
timeout -k 10 120 python tools/diag_div.py 256 0 >> $out 2>&1 || exit 1
timeout -k 10 120 python tools/diag_div.py 32 1 >> $out 2>&1 || exit 1
bash tools/gpu_iter.sh it4
