#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/diag7.log
for v in noalloc alloc poison; do
timeout -k 10 200 python tools/stress_race2.py $v 300 32 >> $O 2>&1 || { echo "FAIL $v rc=$?" >> $O; exit 1; }
done
timeout -k 10 200 python tools/stress_race2.py noalloc 300 2048 >> $O 2>&1 || { echo "FAIL noalloc2048 rc=$?" >> $O; exit 1; }
