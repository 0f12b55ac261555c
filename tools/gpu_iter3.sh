#!/bin/bash
# iteration pass: selected GPU tests, flagship bench, rocprof of the flagship step
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${1:-it}
TESTS=${2:-tests}
timeout -k 10 300 python -u -m pytest $TESTS -m gpu -v -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "EXIT tests $rc" >> gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed rc=$?" >> gpurun_out/${TAG}_bench.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --warmup 10 --no-taxi > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" 2>&1 || exit 1
python3 "$GRAFT_REPO_ROOT/tools/profsum.py" "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof/run_kernel_stats.csv" > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_profsum.txt"
