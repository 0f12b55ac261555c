#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/opt_grid.txt
for G in 256 384 512 768 1024; do
  echo "GRID=$G $(HOPSX_OPT_GRID=$G timeout -k 5 60 python tools/mb_optim.py 2>/dev/null | tail -1)" >> gpurun_out/opt_grid.txt || exit 1
  echo "bench GRID=$G $(HOPSX_OPT_GRID=$G timeout -k 5 120 python bench.py --no-taxi 2>/dev/null | tail -1 | cut -c150-260)" >> gpurun_out/opt_grid.txt || exit 1
done
