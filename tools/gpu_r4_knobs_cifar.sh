#!/bin/bash
# Round-4: env-knob A/B on the CIFAR ResNets (benchmarks/run.py cifar_resnet), each setting twice.
set -o pipefail
out=gpurun_out/${1:-kc}; shift; mkdir -p $out
export TMPDIR=/tmp
ab() { local name=$1 s=$2; shift 2
  r=$(env $s timeout -k 10 240 python benchmarks/run.py "$@" 2>>$out/err.log | tail -1) || { tail $out/err.log; exit 1; }
  echo "[$s] $name $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $out/ab.txt; }
for rep in 1 2; do for s in "" "$@"; do
  ab cifar20 "$s" cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10 --inline
  ab cifar56 "$s" cifar_resnet --depth 56 --batch 128 --steps 50 --warmup 10 --inline
done; done
