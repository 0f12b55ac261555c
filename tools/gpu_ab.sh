#!/bin/bash
# A/B: microbench + flagship bench with the current extension, then with cmp_old/'s build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
SO=hops_examples_amd/_hopsx_ops.cpython-310-x86_64-linux-gnu.so
MB=${MB:-tools/mb_conv.py}
timeout -k 10 120 python -u $MB > gpurun_out/ab_new_mb.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-taxi > gpurun_out/ab_new_bench.log 2>&1 && \
cp cmp_old/$(basename $SO) $SO && \
timeout -k 10 120 python -u $MB > gpurun_out/ab_old_mb.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-taxi > gpurun_out/ab_old_bench.log 2>&1
