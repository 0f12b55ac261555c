#!/bin/bash
# Round-4: persistent data-parallel step (loopback) + deterministic mode evidence on one MI355X.
set -o pipefail
out=gpurun_out/${1:-dp}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_persist_gpu.py tests/test_persist_dp_gpu.py -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -12 $out/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u tools/persist_check.py --timing-only --timing 32 --loopback 2 8 > $out/timing.log 2>&1 || { tail -20 $out/timing.log; exit 1; }
cat $out/timing.log
HOPSX_PERSIST_XFENCE=0 timeout -k 10 200 python -u tools/persist_check.py --timing-only --timing 32 --loopback 8 > $out/timing_nofence.log 2>&1 || { tail -20 $out/timing_nofence.log; exit 1; }
grep "loopback 8" -A14 $out/timing_nofence.log
HOPSX_DETERMINISTIC=1 timeout -k 10 200 python -u tools/det_check.py > $out/det.json 2> $out/det.err || { tail -30 $out/det.err; exit 1; }
cat $out/det.json
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-taxi > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
cat $out/bench.json
HOPSX_DETERMINISTIC=1 timeout -k 10 200 python -u tools/bn_gap.py > $out/bn_gap.txt 2>&1 || { tail -30 $out/bn_gap.txt; exit 1; }
head -80 $out/bn_gap.txt
timeout -k 10 120 python -u tools/dbg_widedeep.py > $out/taxi_phases.txt 2>&1 || { tail -20 $out/taxi_phases.txt; exit 1; }
cat $out/taxi_phases.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/p20 -o run -- python3 benchmarks/run.py cifar_resnet --depth 20 --batch 128 --steps 30 --warmup 10 > $out/p20.log 2>&1 || { tail -20 $out/p20.log; exit 1; }
db=$(find $out/p20 -name '*.db' | head -1); f=$(find $out/p20 -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cp "$f" $out/r20_kernel_stats.csv; [ -n "$db" ] && python tools/profdb.py "$db" > $out/r20_kernels.txt 2>&1; rm -rf $out/p20
head -40 $out/r20_kernels.txt
timeout -k 10 240 python -u -m pytest tests/test_dgrad_par_gpu.py -x -v --timeout 120 --timeout-method thread > $out/dgrad_par.log 2>&1
rc=$?; tail -10 $out/dgrad_par.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/bench_conv_gemm.py --batch 64 --torch > $out/conv_gemm_b64.txt 2>&1 || { tail -20 $out/conv_gemm_b64.txt; exit 1; }
tail -30 $out/conv_gemm_b64.txt
