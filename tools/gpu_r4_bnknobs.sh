#!/bin/bash
# Round-4: BatchNorm launch-geometry knobs (fold deferral by width, grid caps): ResNet A/B on one MI355X.
set -o pipefail
out=gpurun_out/${1:-bnk}; mkdir -p $out
export TMPDIR=/tmp
ab() { local name=$1 s=$2; shift 2
  r=$(env $s timeout -k 10 240 python benchmarks/run.py "$@" 2>>$out/err.log | tail -1) || { tail $out/err.log; exit 1; }
  echo "[$s] $name $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $out/ab.txt; }
for s in "" "HOPSX_DISABLE=bn_defer" "HOPSX_BN_DEFER_MAXC=512" "HOPSX_BN_DEFER_MAXC=256" "HOPSX_BN_APPLY_MAXG=2048" "HOPSX_BN_APPLY_MAXG=8192" "HOPSX_BN_MAXG=2048" "HOPSX_BN_MAXG=512"; do
  ab r50_b64 "$s" resnet50 --batch 64 --steps 30 --warmup 5
done
for s in "" "HOPSX_DISABLE=bn_defer" "HOPSX_BN_MAXG=2048" "HOPSX_BN_APPLY_MAXG=2048"; do
  ab cifar20 "$s" cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10
done
