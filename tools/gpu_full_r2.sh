#!/bin/bash
# full GPU test suite + smoke, then every BASELINE config (benchmarks/run.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 && \
bash tools/gpu_bench_all_r2.sh
rc=$?
echo "EXIT $rc" >> gpurun_out/pytest_gpu.log
exit $rc
