#!/bin/bash
set -o pipefail
out=gpurun_out/r3e; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_widedeep_fused_gpu.py -x -q --timeout 120 --timeout-method thread > $out/wd_tests.log 2>&1 || { tail -30 $out/wd_tests.log; exit 1; }
tail -2 $out/wd_tests.log
timeout -k 10 120 python benchmarks/run.py taxi --steps 2000 --warmup 50 > $out/taxi.json 2>&1 || exit $?
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $out/bench.json 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof256 -o run -- python benchmarks/run.py resnet50 --batch 256 --steps 4 --warmup 2 > $out/prof256.log 2>&1 || exit $?
grep '^{' $out/taxi.json $out/bench.json | cut -c1-400
