set -o pipefail
o=gpurun_out/${1:-r5_r20knobs}; mkdir -p $o; export TMPDIR=/tmp
run() { env $1 timeout -k 10 200 python benchmarks/run.py cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10 > $o/r.json 2> $o/err.log || { tail -20 $o/err.log; exit 1; }
  echo "[$1] $(python -c "import json; r=json.loads(open('$o/r.json').read().strip().splitlines()[-1]); print(r['value'], r['ms_per_step'])")"; }
for k in X=0 HOPSX_BN_APPLY_MAXG=256 HOPSX_BN_APPLY_MAXG=128 HOPSX_BN_RPT=8 HOPSX_BN_MAXG=512 HOPSX_GEMM_T64_MIN=256 HOPSX_GEMM_T128_MIN=128 HOPSX_WGRAD_MFMA_MAXK=288 X=0; do run $k; done
