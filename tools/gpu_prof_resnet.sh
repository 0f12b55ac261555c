#!/bin/bash
# ResNet benchmarks + rocprofv3 kernel tables (run through gpurun from the repo root).
# usage: tools/gpu_prof_resnet.sh <tag>
set -o pipefail
tag=${1:-r3}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 150 python benchmarks/run.py cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10 > $out/cifar20.json 2> $out/cifar20.err || exit $?
timeout -k 10 150 python benchmarks/run.py cifar_resnet --depth 56 --batch 128 --steps 50 --warmup 10 > $out/cifar56.json 2> $out/cifar56.err || exit $?
timeout -k 10 200 python benchmarks/run.py resnet50 --batch 64 --steps 30 --warmup 5 > $out/r50_b64.json 2> $out/r50_b64.err || exit $?
timeout -k 10 300 python benchmarks/run.py resnet50 --batch 256 --steps 10 --warmup 3 > $out/r50_b256.json 2> $out/r50_b256.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof20 -o run -- python benchmarks/run.py cifar_resnet --depth 20 --batch 128 --steps 50 --warmup 10 > $out/prof20.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof50 -o run -- python benchmarks/run.py resnet50 --batch 64 --steps 20 --warmup 5 > $out/prof50.log 2>&1 || exit $?
for d in prof20 prof50; do f=$(find $out/$d -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $out/${d}_kernel_stats.csv; done
cat $out/*.json
