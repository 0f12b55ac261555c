#!/bin/bash
# Round-4: BN backward act' mask from z (no y read): numerics, then ResNet A/B (HOPSX_DISABLE=bn_zmask).
set -o pipefail
out=gpurun_out/${1:-zmask}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_bnstats_gpu.py tests/test_models_gpu.py tests/test_proj_addend_gpu.py tests/test_stem_pad_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -4 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
ab() { local name=$1 s=$2; shift 2
  r=$(env $s timeout -k 10 240 python benchmarks/run.py "$@" 2>>$out/err.log | tail -1) || { tail $out/err.log; exit 1; }
  echo "[$s] $name $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $out/ab.txt; }
for s in "" "HOPSX_DISABLE=bn_zmask" "" "HOPSX_DISABLE=bn_zmask"; do ab r50_b64 "$s" resnet50 --batch 64 --steps 30 --warmup 5; done
for s in "" "HOPSX_DISABLE=bn_zmask"; do ab cifar20 "$s" cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10; ab cifar56 "$s" cifar_resnet --depth 56 --batch 128 --steps 50 --warmup 10; done
ab r50_b256 "" resnet50 --batch 256 --steps 10 --warmup 3
