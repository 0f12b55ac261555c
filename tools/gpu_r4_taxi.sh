#!/bin/bash
# Chicago-taxi fused step on one MI355X: its GPU tests, phase stamps, the benchmark at 200 steps and
# at the driver's bench.py setting.
set -o pipefail
tag=${1:-t}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_widedeep_fused_gpu.py tests/test_tfx_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -4 $out/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 180 python -u tools/dbg_widedeep.py > $out/phases.txt 2>&1 || { tail -20 $out/phases.txt; exit 1; }
cat $out/phases.txt
timeout -k 10 180 python -u benchmarks/run.py taxi --steps 200 --warmup 20 > $out/taxi.json 2> $out/taxi.err || { tail $out/taxi.err; exit 1; }
cat $out/taxi.json
timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
cat $out/bench.json
