#!/bin/bash
# Round-4: 8-channel image stems + weight-gradient routing knobs: numerics, then ResNet A/B.
set -o pipefail
out=gpurun_out/${1:-stem}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_stem_pad_gpu.py tests/test_debug_checks_gpu.py tests/test_models_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -4 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
ab() { local name=$1 s=$2; shift 2
  r=$(env $s timeout -k 10 240 python benchmarks/run.py "$@" 2>>$out/err.log | tail -1) || { tail $out/err.log; exit 1; }
  echo "[$s] $name $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $out/ab.txt; }
for s in "" "HOPSX_DISABLE=stem_pad" "HOPSX_WGRAD_MFMA_MAX_MK=1000000000000"; do
  ab r50_b64 "$s" resnet50 --batch 64 --steps 30 --warmup 5
done
for s in "" "HOPSX_DISABLE=stem_pad"; do
  ab cifar20 "$s" cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10; ab cifar56 "$s" cifar_resnet --depth 56 --batch 128 --steps 50 --warmup 10
done
ab r50_b256 "" resnet50 --batch 256 --steps 10 --warmup 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/p50 -o run -- python3 benchmarks/run.py resnet50 --batch 64 --steps 20 --warmup 5 > $out/p50.log 2>&1 || { tail -20 $out/p50.log; exit 1; }
db=$(find $out/p50 -name '*.db' | head -1); python tools/profdb.py "$db" > $out/r50_b64_kernels.txt 2>&1; rm -rf $out/p50; head -32 $out/r50_b64_kernels.txt | cut -c1-180
