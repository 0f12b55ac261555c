#!/bin/bash
# Round-4: env-knob A/B on ResNet-50 B=64 / B=256 (benchmarks/run.py), each setting twice.
set -o pipefail
out=gpurun_out/${1:-k50}; shift; mkdir -p $out
export TMPDIR=/tmp
ab() { local name=$1 s=$2; shift 2
  r=$(env $s timeout -k 10 240 python benchmarks/run.py "$@" 2>>$out/err.log | tail -1) || { tail $out/err.log; exit 1; }
  echo "[$s] $name $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $out/ab.txt; }
for rep in 1 2; do for s in "" "$@"; do ab r50_b64 "$s" resnet50 --batch 64 --steps 30 --warmup 5; done; done
for s in "" "$@"; do ab r50_b256 "$s" resnet50 --batch 256 --steps 10 --warmup 3; done
