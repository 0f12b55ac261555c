#!/bin/bash
# A/B of env knobs on the flagship bench (MNIST only, 400 steps), one line per setting.
# usage: tools/gpu_knobs.sh <tag> "ENV=1 ENV2=2" "ENV=3" ...   ("" = baseline)
set -o pipefail
tag=${1:-k}
shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for s in "$@"; do
  r=$(env $s timeout -k 10 120 python bench.py --steps 400 --warmup 40 --no-taxi 2>>$out/err.log) || { echo "FAIL [$s]"; tail -5 $out/err.log; exit 1; }
  echo "[$s] $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a $out/ab.txt
done
exit 0
