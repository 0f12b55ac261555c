#!/bin/bash
# Python-side routing knobs A/B on ResNet-50 / ResNet-20: side-stream wgrad threshold, 1x1 routing.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B="timeout -k 10 200 python -u benchmarks/run.py"
: > gpurun_out/knobs.txt
for cfg in "resnet50 --batch 8" "resnet50 --batch 64" "cifar_resnet"; do
  echo "default $cfg :: $($B $cfg --steps 20 --warmup 5 | tail -1 | cut -c60-140)" >> gpurun_out/knobs.txt || exit 1
  echo "par1e9 $cfg :: $(HOPSX_PAR_WGRAD_MIN_FLOP=1e9 $B $cfg --steps 20 --warmup 5 | tail -1 | cut -c60-140)" >> gpurun_out/knobs.txt || exit 1
  echo "par8e9 $cfg :: $(HOPSX_PAR_WGRAD_MIN_FLOP=8e9 $B $cfg --steps 20 --warmup 5 | tail -1 | cut -c60-140)" >> gpurun_out/knobs.txt || exit 1
  echo "flop3e7 $cfg :: $(HOPSX_BNSTATS_MAX_1X1_FLOP=3e7 $B $cfg --steps 20 --warmup 5 | tail -1 | cut -c60-140)" >> gpurun_out/knobs.txt || exit 1
  echo "px64 $cfg :: $(HOPSX_PLAIN_MIN_PX=64 $B $cfg --steps 20 --warmup 5 | tail -1 | cut -c60-140)" >> gpurun_out/knobs.txt || exit 1
done
