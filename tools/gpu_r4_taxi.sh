#!/bin/bash
# Chicago-taxi fused step on one MI355X: phase stamps + the benchmark at the driver's setting.
set -o pipefail
tag=${1:-t}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 180 python -u tools/dbg_widedeep.py > $out/phases.txt 2>&1 || { tail -20 $out/phases.txt; exit 1; }
cat $out/phases.txt
timeout -k 10 180 python -u benchmarks/run.py taxi --steps 200 --warmup 20 > $out/taxi.json 2> $out/taxi.err || { tail $out/taxi.err; exit 1; }
cat $out/taxi.json
