#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/diag6.log
timeout -k 10 300 python tools/stress_race.py 20000 32 graph >> $O 2>&1 || { echo "FAIL graph rc=$?" >> $O; exit 1; }
timeout -k 10 300 python tools/stress_race.py 5000 32 eager >> $O 2>&1 || { echo "FAIL eager rc=$?" >> $O; exit 1; }
timeout -k 10 300 python tools/stress_race.py 10000 256 graph >> $O 2>&1 || { echo "FAIL g256 rc=$?" >> $O; exit 1; }
timeout -k 10 300 python tools/stress_race.py 3000 2048 graph >> $O 2>&1 || { echo "FAIL g2048 rc=$?" >> $O; exit 1; }
