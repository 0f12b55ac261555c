#!/bin/bash
# steps_per_execution A/B on the flagship bench at the driver's K=20/W=5 and at 200 steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/spe.txt
for spe in 8 16 32; do
  for k in "--steps 20 --warmup 5" "--steps 200 --warmup 20"; do
    echo "spe=$spe $k :: $(HOPSX_STEPS_PER_EXEC=$spe timeout -k 10 200 python -u bench.py $k | tail -1 | cut -c60-260)" >> gpurun_out/spe.txt || exit 1
  done
done
