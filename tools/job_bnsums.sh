set -o pipefail
o=gpurun_out/${1:-r5_bnsums}; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bn_dgrad_sums_gpu.py tests/test_bnstats_gpu.py > $o/t.log 2>&1 || { tail -40 $o/t.log; exit 1; }
tail -3 $o/t.log
for d in bn_dgrad_sums "" bn_dgrad_sums ""; do
  HOPSX_DISABLE=$d timeout -k 10 200 python benchmarks/run.py cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10 > $o/r20_$d.json 2> $o/r20_err.log || { tail -20 $o/r20_err.log; exit 1; }
  echo "[$d] $(python -c "import json,sys; r=json.loads(open('$o/r20_$d.json').read().strip().splitlines()[-1]); print(r['value'], r['ms_per_step'])")"
done
