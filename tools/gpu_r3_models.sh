#!/bin/bash
# GPU tests of this round's kernels + model benchmarks (titanic ingest, ResNet-50 B=64/256, CIFAR).
set -o pipefail
tag=${1:-m}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad_glds_gpu.py tests/test_parquet_reader.py > $out/test.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/run.py titanic --steps 100 --warmup 10 > $out/titanic1.json 2> $out/titanic1.err || exit $?
timeout -k 10 200 python benchmarks/run.py resnet50 --batch 64 --steps 30 --warmup 5 > $out/r50_b64.json 2> $out/r50_b64.err || exit $?
timeout -k 10 300 python benchmarks/run.py resnet50 --batch 256 --steps 10 --warmup 3 > $out/r50_b256.json 2> $out/r50_b256.err || exit $?
timeout -k 10 150 python benchmarks/run.py cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10 > $out/cifar20.json 2> $out/cifar20.err || exit $?
timeout -k 10 150 python benchmarks/run.py cifar_resnet --depth 56 --batch 128 --steps 50 --warmup 10 > $out/cifar56.json 2> $out/cifar56.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof50 -o run -- python benchmarks/run.py resnet50 --batch 64 --steps 20 --warmup 5 > $out/prof50.log 2>&1 || exit $?
exit 0
