#!/bin/bash
# Persistent flagship step on one MI355X (run through gpurun from the repo root): numerics vs the
# fp64 reference + phase timing, its GPU tests, then bench.py at the driver's setting.
# usage: tools/gpu_persist.sh <tag>
set -o pipefail
tag=${1:-p}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/persist_check.py --steps 8 --timing 32 > $out/check.log 2>&1
rc=$?; cat $out/check.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_persist_gpu.py -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -15 $out/pytest.log
# 1 = a test assertion failed (the GPU is fine): still measure; anything else stops here
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-taxi > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 180 python bench.py --steps 200 --warmup 20 --no-taxi > $out/bench200.json 2> $out/bench200.err || { tail $out/bench200.err; exit 1; }
cat $out/bench200.json
