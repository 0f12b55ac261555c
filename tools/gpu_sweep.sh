#!/bin/bash
# bench sweep over one env variable: VAR v1 v2 ... -> gpurun_out/sweep_VAR.txt
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
VAR=$1; shift
out=gpurun_out/sweep_${VAR}.txt
: > $out
for v in "$@"; do
  env "$VAR=$v" timeout -k 10 120 python bench.py --steps 400 --warmup 30 > gpurun_out/sweep_tmp.log 2>&1 || { echo "$v FAILED" >> $out; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sweep_tmp.log | tr '\n' ' ')" >> $out
done
