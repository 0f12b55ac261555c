set -o pipefail
o=gpurun_out/${1:-r5_bnknobs}; mkdir -p $o; export TMPDIR=/tmp
run() { env $1 timeout -k 10 200 python benchmarks/run.py resnet50 --batch 64 --steps 12 --warmup 4 > $o/r.json 2> $o/err.log || { tail -20 $o/err.log; exit 1; }
  echo "[$1] $(python -c "import json; r=json.loads(open('$o/r.json').read().strip().splitlines()[-1]); print(r['value'], r['ms_per_step'])")"; }
for k in X=0 HOPSX_BN_APPLY_MAXG=1024 HOPSX_BN_APPLY_MAXG=2048 HOPSX_BN_APPLY_MAXG=16384 HOPSX_BN_FOLD_MINC=256 HOPSX_BN_FOLD_MINC=64 X=0; do run $k; done
