#!/bin/bash
# conv kernel iteration: kernel GPU tests, microbench + phase stamps, flagship bench, A/B vs cmp_old
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
SO=hops_examples_amd/_hopsx_ops.cpython-310-x86_64-linux-gnu.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_kernels_v2_gpu.py tests/test_train_gpu.py tests/test_graph_replay_gpu.py \
  > gpurun_out/ci_tests.log 2>&1 && \
timeout -k 10 120 python -u tools/mb_conv.py > gpurun_out/ci_mb.log 2>&1 && \
timeout -k 10 120 python -u tools/dbg_convfwd.py > gpurun_out/ci_dbg.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-taxi > gpurun_out/ci_bench.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-taxi > gpurun_out/ci_bench20.log 2>&1 && \
if [ -f cmp_old/$(basename $SO) ]; then cp cmp_old/$(basename $SO) $SO && \
  timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-taxi > gpurun_out/ci_bench_old.log 2>&1; fi
