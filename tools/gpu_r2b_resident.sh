#!/bin/bash
# Benchmark harness: HBM-resident batches + steps_per_execution graphs (HOPSX_BENCH_RESIDENT=1) vs
# per-step input copies and one graph per step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B="timeout -k 10 200 python -u benchmarks/run.py"
: > gpurun_out/resident.txt
for cfg in "cifar_resnet" "cifar_resnet --depth 56" "resnet50 --batch 8" "resnet50 --batch 64" "taxi" "titanic"; do
  echo "copy $cfg :: $($B $cfg --steps 30 --warmup 10 | tail -1 | cut -c1-170)" >> gpurun_out/resident.txt || exit 1
  echo "resident $cfg :: $(HOPSX_BENCH_RESIDENT=1 $B $cfg --steps 30 --warmup 10 | tail -1 | cut -c1-170)" >> gpurun_out/resident.txt || exit 1
done
