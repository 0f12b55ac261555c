set -o pipefail
o=gpurun_out/${1:-r5_bnval}; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_bnstats_gpu.py tests/test_bn_dgrad_sums_gpu.py tests/test_kernels_gpu.py tests/test_deterministic_gpu.py > $o/t.log 2>&1 || { grep -E "FAIL|Error|assert" $o/t.log | tail -20; exit 1; }
tail -1 $o/t.log
run() { env $1 timeout -k 10 200 python benchmarks/run.py $2 > $o/r.json 2> $o/err.log || { tail -20 $o/err.log; exit 1; }
  echo "[$1] $2 -> $(python -c "import json; r=json.loads(open('$o/r.json').read().strip().splitlines()[-1]); print(r['value'], r['ms_per_step'])")"; }
run X=0 "resnet50 --batch 64 --steps 30 --warmup 5"
run X=0 "resnet50 --batch 256 --steps 10 --warmup 3"
run X=0 "cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10"
run X=0 "cifar_resnet --depth 56 --batch 128 --steps 60 --warmup 10"
