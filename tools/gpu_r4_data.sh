#!/bin/bash
# Round-4 data path + teardown checks on one MI355X (through gpurun from the repo root):
# GB-scale Parquet -> HBM ingest, the Titanic config-4 bench, and 2 / 4-rank rehearsals that exit
# through normal interpreter teardown (HOPSX_RANK_FAST_EXIT=0, faulthandler on) to catch the abort.
# usage: tools/gpu_r4_data.sh <tag>
set -o pipefail
tag=${1:-d}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u benchmarks/run.py titanic_ingest --rows 50000000 > $out/ingest.json 2> $out/ingest.err || { tail -20 $out/ingest.err; exit 1; }
cat $out/ingest.json
timeout -k 10 300 python -u benchmarks/run.py titanic --rows 891000 --steps 300 --warmup 20 > $out/titanic.json 2> $out/titanic.err || { tail -20 $out/titanic.err; exit 1; }
cat $out/titanic.json
for n in 2 4; do
  HOPSX_RANK_FAST_EXIT=0 PYTHONFAULTHANDLER=1 timeout -k 10 240 python -u bench.py --gpus $n --rehearse --steps 5 --warmup 2 --no-taxi > $out/rh$n.json 2> $out/rh$n.err
  rc=$?
  echo "rehearsal $n ranks rc=$rc"; tail -3 $out/rh$n.json
  grep -n -i "terminate\|abort\|Fatal Python\|Segmentation" $out/rh$n.err | head -20
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || [ $rc -eq 134 ] || [ $rc -eq 250 ] || exit $rc
done
