#!/bin/bash
# Flagship (MNIST E3 step) check on one MI355X: targeted GPU tests, bench.py, rocprofv3 kernel table.
# usage: tools/gpu_flagship.sh <tag> [test files...]
set -o pipefail
tag=${1:-f}
shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread "$@" > $out/test.log 2>&1 || { tail -40 $out/test.log; exit 1; }
  tail -2 $out/test.log
fi
timeout -k 10 120 python bench.py --steps 200 --warmup 20 > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $out/bench20.json 2>> $out/bench.err || { tail $out/bench.err; exit 1; }
cat $out/bench.json $out/bench20.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python bench.py --steps 100 --warmup 20 --no-taxi > $out/prof.log 2>&1 || { tail $out/prof.log; exit 1; }
f=$(find $out/prof -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $out/kernel_stats.csv && python tools/kstats.py $out/kernel_stats.csv 2>/dev/null | head -20
exit 0
