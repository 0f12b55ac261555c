#!/bin/bash
# Round-4: gg vectorized epilogue + Bottleneck shortcut-gradient fusion: numerics, conv GEMM table, ResNet-50 A/B.
set -o pipefail
out=gpurun_out/${1:-vec}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_kernels_v2_gpu.py tests/test_models_gpu.py tests/test_dgrad_par_gpu.py tests/test_wgrad_glds_gpu.py tests/test_bnstats_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -4 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_conv_gemm.py --batch 64 --torch > $out/conv_gemm_b64.txt 2>&1 || { tail -20 $out/conv_gemm_b64.txt; exit 1; }
tail -1 $out/conv_gemm_b64.txt
for s in "" "HOPSX_DISABLE=res_addend"; do
  r=$(env $s timeout -k 10 200 python benchmarks/run.py resnet50 --batch 64 --steps 30 --warmup 5 2>>$out/err.log | tail -1) || { tail $out/err.log; exit 1; }
  echo "[$s] b64 $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
r=$(timeout -k 10 300 python benchmarks/run.py resnet50 --batch 256 --steps 10 --warmup 3 2>>$out/err.log | tail -1) || { tail $out/err.log; exit 1; }
echo "b256 $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
