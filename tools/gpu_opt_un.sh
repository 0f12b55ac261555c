#!/bin/bash
# optimizer unroll/grid sweep at the flagship arena size, then the flagship bench with the default pick
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/opt_un.txt
for UN in 3 6; do for G in 128 256 512; do
  echo "UN=$UN GRID=$G $(HOPSX_OPT_UN=$UN HOPSX_OPT_GRID=$G timeout -k 5 60 python tools/mb_optim.py 2>/dev/null | tail -1)" >> gpurun_out/opt_un.txt || exit 1
done; done
for UN in 3 6; do
  echo "bench UN=$UN $(HOPSX_OPT_UN=$UN timeout -k 5 120 python bench.py --no-taxi 2>/dev/null | tail -1 | cut -c1-200)" >> gpurun_out/opt_un.txt || exit 1
done
