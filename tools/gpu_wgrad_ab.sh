#!/bin/bash
# glds weight-gradient kernel: numerics, then ResNet-50 A/B (HOPSX_DISABLE=wgrad_glds) and a profile.
# usage (through gpurun, repo root): tools/gpu_wgrad_ab.sh <tag>
set -o pipefail
tag=${1:-wg}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wgrad_glds_gpu.py > $out/test.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/run.py resnet50 --batch 64 --steps 30 --warmup 5 > $out/r50_b64.json 2> $out/r50_b64.err || exit $?
HOPSX_DISABLE=wgrad_glds timeout -k 10 200 python benchmarks/run.py resnet50 --batch 64 --steps 30 --warmup 5 > $out/r50_b64_off.json 2> $out/r50_b64_off.err || exit $?
timeout -k 10 300 python benchmarks/run.py resnet50 --batch 256 --steps 10 --warmup 3 > $out/r50_b256.json 2> $out/r50_b256.err || exit $?
HOPSX_WGRAD_GLDS_FIRST=1 timeout -k 10 200 python benchmarks/run.py resnet50 --batch 64 --steps 30 --warmup 5 > $out/r50_b64_first.json 2> $out/r50_b64_first.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof50 -o run -- python benchmarks/run.py resnet50 --batch 64 --steps 20 --warmup 5 > $out/prof50.log 2>&1 || exit $?
f=$(find $out/prof50 -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $out/prof50_kernel_stats.csv
cat $out/*.json
