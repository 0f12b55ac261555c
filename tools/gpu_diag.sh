#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/diag8.log
timeout -k 10 300 python tools/stress_race.py 20000 32 graph >> $O 2>&1 || { echo "FAIL graph32 rc=$?" >> $O; exit 1; }
timeout -k 10 300 python tools/stress_race.py 10000 256 graph >> $O 2>&1 || { echo "FAIL graph256 rc=$?" >> $O; exit 1; }
for v in noalloc alloc; do
timeout -k 10 200 python tools/stress_race2.py $v 2000 32 >> $O 2>&1 || { echo "FAIL $v rc=$?" >> $O; exit 1; }
done
timeout -k 10 200 python bench.py >> $O 2>&1 || { echo "FAIL bench rc=$?" >> $O; exit 1; }
timeout -k 10 200 python bench.py --batch-per-gpu 256 --no-taxi >> $O 2>&1 || { echo "FAIL bench256 rc=$?" >> $O; exit 1; }
