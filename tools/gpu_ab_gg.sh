set -o pipefail
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels_v2_gpu.py tests/test_bnstats_gpu.py tests/test_models_gpu.py 2>&1 | tail -2
for s in "" "HOPSX_GG_MIN_N=0" "" "HOPSX_GG_MIN_N=0"; do
  a=$(env $s timeout -k 10 200 python benchmarks/run.py resnet50 --batch 64 --steps 20 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'])")
  b=$(env $s timeout -k 10 200 python benchmarks/run.py resnet50 --batch 256 --steps 8 --warmup 3 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'])")
  c=$(env $s timeout -k 10 200 python benchmarks/run.py cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'])")
  echo "[$s] r50_b64 $a r50_b256 $b r20 $c"
done
