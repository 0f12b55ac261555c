#!/bin/bash
# driver-style flagship runs (bench.py --steps 20 --warmup 5, MNIST only), alternating settings
# usage: tools/gpu_ab20.sh <tag> <reps> "ENV=.." "ENV=.." ...
set -o pipefail
tag=${1:-a}; reps=${2:-3}; shift 2
out=gpurun_out/$tag; mkdir -p $out
for i in $(seq $reps); do
  for s in "$@"; do
    r=$(env $s timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-taxi 2>>$out/err.log) || { echo "FAIL [$s]"; exit 1; }
    echo "[$s] $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a $out/ab.txt
  done
done
exit 0
