#!/bin/bash
# perf iteration: kernel/graph GPU tests, flagship bench, rocprofv3 kernel stats of the flagship step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_train_gpu.py tests/test_graph_replay_gpu.py tests/test_kernels_gpu.py tests/test_kernels_fused_gpu.py tests/test_p2p_gpu.py \
  > gpurun_out/iter_tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py > gpurun_out/iter_bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/iter_prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 100 --warmup 20 --no-taxi > "$R/gpurun_out/iter_prof.log" 2>&1
rc=$?
echo "EXIT $rc" >> "$R/gpurun_out/iter_bench.log"
exit $rc
