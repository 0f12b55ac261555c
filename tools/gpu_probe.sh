#!/bin/bash
# Taxi fused-step phases + ResNet-20 / ResNet-50 kernel tables (one MI355X).
set -o pipefail
out=gpurun_out/${1:-p}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python tools/dbg_widedeep.py > $out/widedeep_phases.txt 2>&1 || { tail $out/widedeep_phases.txt; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof20 -o run -- python benchmarks/run.py cifar_resnet --depth 20 --batch 128 --steps 50 --warmup 10 > $out/prof20.log 2>&1 || { tail $out/prof20.log; exit 1; }
python tools/profdb.py $out/prof20/run_results.db > $out/r20_kern.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof50 -o run -- python benchmarks/run.py resnet50 --batch 64 --steps 20 --warmup 5 > $out/prof50.log 2>&1 || { tail $out/prof50.log; exit 1; }
python tools/profdb.py $out/prof50/run_results.db > $out/r50_kern.txt
rm -rf $out/prof20 $out/prof50
cat $out/widedeep_phases.txt; head -25 $out/r20_kern.txt; head -25 $out/r50_kern.txt
