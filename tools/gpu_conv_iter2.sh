#!/bin/bash
# quick conv iteration: kernel tests, stamps, VALU counters, flagship bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_kernels_v2_gpu.py tests/test_train_gpu.py > gpurun_out/ci_tests.log 2>&1 && \
timeout -k 10 120 python -u tools/mb_conv.py > gpurun_out/ci_mb.log 2>&1 && \
timeout -k 10 120 python -u tools/dbg_convfwd.py > gpurun_out/ci_dbg.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-taxi > gpurun_out/ci_bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH -d "$R/gpurun_out/pmc_c5" -o run --output-format csv -- python3 "$R/tools/mb_conv.py" > "$R/gpurun_out/pmc_5.log" 2>&1
