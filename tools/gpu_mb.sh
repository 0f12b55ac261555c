#!/bin/bash
# targeted tests + kernel-level microbench under rocprof (kernel time only)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-mb}; TESTS=${2:-tests/test_kernels_v2_gpu.py}; ONLY=${3:-}
timeout -k 10 300 python -u -m pytest $TESTS -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "EXIT tests $rc" >> gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for V in ${CPWS:-0}; do
  HOPSX_WGRAD_CPW=$V MB_ONLY=$ONLY timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_kt$V" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/microbench.py" 32 200 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_kt$V.log" 2>&1 || exit 1
  python3 "$GRAFT_REPO_ROOT/tools/profsum.py" "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_kt$V/run_kernel_stats.csv" 1 12 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_kt$V.txt"
done
