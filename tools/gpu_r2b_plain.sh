#!/bin/bash
# 1x1 conv routing A/B (Python-side knobs): library GEMM floor in pixels, BN-stats epilogue FLOP cap.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B="timeout -k 10 200 python -u benchmarks/run.py"
: > gpurun_out/plain.txt
for cfg in "resnet50 --batch 8" "resnet50 --batch 64"; do
  echo "default $cfg :: $($B $cfg --steps 20 --warmup 5 | tail -1 | cut -c60-140)" >> gpurun_out/plain.txt || exit 1
  echo "px256+flop1e8 $cfg :: $(HOPSX_PLAIN_MIN_PX=256 HOPSX_BNSTATS_MAX_1X1_FLOP=1e8 $B $cfg --steps 20 --warmup 5 | tail -1 | cut -c60-140)" >> gpurun_out/plain.txt || exit 1
  echo "px256 $cfg :: $(HOPSX_PLAIN_MIN_PX=256 $B $cfg --steps 20 --warmup 5 | tail -1 | cut -c60-140)" >> gpurun_out/plain.txt || exit 1
  echo "flop1e8 $cfg :: $(HOPSX_BNSTATS_MAX_1X1_FLOP=1e8 $B $cfg --steps 20 --warmup 5 | tail -1 | cut -c60-140)" >> gpurun_out/plain.txt || exit 1
  echo "flop1e10 $cfg :: $(HOPSX_BNSTATS_MAX_1X1_FLOP=1e10 $B $cfg --steps 20 --warmup 5 | tail -1 | cut -c60-140)" >> gpurun_out/plain.txt || exit 1
done
