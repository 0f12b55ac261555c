#!/bin/bash
# Full round-end style verification on one MI355X (run through gpurun from the repo root):
# GPU test suite, smoke(), default bench.py, ResNet/taxi model benches.
# usage: tools/gpu_verify.sh <tag> [quick]
set -o pipefail
tag=${1:-v}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 1; }
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
cat $out/smoke.log $out/bench.json
[ "$2" = quick ] && exit 0
timeout -k 10 150 python benchmarks/run.py cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10 > $out/cifar20.json 2> $out/cifar20.err || exit $?
timeout -k 10 200 python benchmarks/run.py resnet50 --batch 64 --steps 30 --warmup 5 > $out/r50_b64.json 2> $out/r50_b64.err || exit $?
timeout -k 10 300 python benchmarks/run.py resnet50 --batch 256 --steps 10 --warmup 3 > $out/r50_b256.json 2> $out/r50_b256.err || exit $?
cat $out/cifar20.json $out/r50_b64.json $out/r50_b256.json
exit 0
