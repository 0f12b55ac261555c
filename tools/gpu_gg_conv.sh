#!/bin/bash
# gg engine: numerics, then the per-layer conv GEMM table with and without it (+ PyTorch), B=64.
set -o pipefail
tag=${1:-ggc}; B=${2:-64}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad_glds_gpu.py tests/test_parquet_reader.py > $out/test.log 2>&1 || exit $?
timeout -k 10 150 python tools/bench_conv_gemm.py --batch $B --torch > $out/gg_on.jsonl 2>&1 || exit $?
HOPSX_DISABLE=gg timeout -k 10 150 python tools/bench_conv_gemm.py --batch $B > $out/gg_off.jsonl 2>&1 || exit $?
timeout -k 10 200 python benchmarks/run.py titanic --steps 100 --warmup 10 > $out/titanic1.json 2> $out/titanic1.err || exit $?
exit 0
