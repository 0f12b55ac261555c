#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for G in 256 512 1024 2048; do
  HOPSX_OPT_GRID=$G timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/opt_$G" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/mb_optim.py" >> "$GRAFT_REPO_ROOT/gpurun_out/opt.log" 2>&1 || exit 1
  echo "G=$G $(python3 $GRAFT_REPO_ROOT/tools/profsum.py $GRAFT_REPO_ROOT/gpurun_out/opt_$G/run_kernel_stats.csv 1 2 | tail -1)" >> "$GRAFT_REPO_ROOT/gpurun_out/opt.txt"
done
