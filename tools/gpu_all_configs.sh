#!/bin/bash
# Every BASELINE config's benchmark once on one MI355X (benchmarks/run.py), JSON lines to gpurun_out/<tag>/all.jsonl
set -o pipefail
out=gpurun_out/${1:-c}; mkdir -p $out; : > $out/all.jsonl
run() { timeout -k 10 300 python benchmarks/run.py "$@" 2>>$out/err.log | tail -1 >> $out/all.jsonl || { echo "FAIL $*"; tail -5 $out/err.log; exit 1; }; }
timeout -k 10 300 python benchmarks/run.py mnist_launch_cpu --steps 20 --warmup 2 2>>$out/err.log | tail -1 >> $out/all.jsonl || true
run mnist_mirrored --steps 200 --warmup 20
run taxi --steps 200 --warmup 20
run taxi --steps 200 --warmup 20 --from-transform
run titanic --steps 200 --warmup 20
run cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10
run cifar_resnet --depth 56 --batch 128 --steps 50 --warmup 10
run resnet50 --batch 8 --steps 30 --warmup 5
cut -c1-260 $out/all.jsonl
