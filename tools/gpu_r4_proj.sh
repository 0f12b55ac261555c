#!/bin/bash
# Round-4: projection-shortcut gradient hand-off: numerics, ResNet A/B, ResNet-20 + ResNet-50 kernel tables.
set -o pipefail
out=gpurun_out/${1:-proj}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_proj_addend_gpu.py tests/test_models_gpu.py tests/test_kernels_gpu.py tests/test_bnstats_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -4 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
ab() { local name=$1 s=$2; shift 2
  r=$(env $s timeout -k 10 240 python benchmarks/run.py "$@" 2>>$out/err.log | tail -1) || { tail $out/err.log; exit 1; }
  echo "[$s] $name $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $out/ab.txt; }
for s in "" "HOPSX_DISABLE=proj_addend"; do ab r50_b64 "$s" resnet50 --batch 64 --steps 30 --warmup 5; done
for s in "" "HOPSX_DISABLE=proj_addend"; do ab cifar20 "$s" cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10; done
kt() { local d=$1 name=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$d -o run -- python3 "$@" > $out/$d.log 2>&1 || { tail -20 $out/$d.log; exit 1; }
  db=$(find $out/$d -name '*.db' | head -1); python tools/profdb.py "$db" > $out/$name 2>&1; rm -rf $out/$d; head -14 $out/$name | cut -c1-170; }
kt p20 r20_kernels.txt benchmarks/run.py cifar_resnet --depth 20 --batch 128 --steps 50 --warmup 10 --inline
kt p50 r50_b64_kernels.txt benchmarks/run.py resnet50 --batch 64 --steps 20 --warmup 5
