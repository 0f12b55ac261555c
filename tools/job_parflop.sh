set -o pipefail
o=gpurun_out/${1:-r5_parflop}; mkdir -p $o; export TMPDIR=/tmp
run() { env $1 timeout -k 10 200 python benchmarks/run.py $2 > $o/r.json 2> $o/err.log || { tail -20 $o/err.log; exit 1; }
  echo "[$1] $2 -> $(python -c "import json; r=json.loads(open('$o/r.json').read().strip().splitlines()[-1]); print(r['value'], r['ms_per_step'])")"; }
for k in X=0 HOPSX_PAR_WGRAD_MIN_FLOP=5e9 HOPSX_PAR_WGRAD_MIN_FLOP=2e10 HOPSX_PAR_WGRAD_MIN_FLOP=1e12 X=0 HOPSX_PAR_WGRAD_MIN_FLOP=2e10; do run $k "resnet50 --batch 64 --steps 12 --warmup 4"; done
for k in X=0 HOPSX_PAR_WGRAD_MIN_FLOP=2e10 HOPSX_PAR_WGRAD_MIN_FLOP=1e12; do run $k "resnet50 --batch 256 --steps 8 --warmup 3"; done
for k in HOPSX_PAR_WGRAD_MIN_FLOP=5e9 HOPSX_PAR_WGRAD_MIN_FLOP=1e12; do run $k "resnet50 --batch 8 --steps 30 --warmup 5"; done
for k in X=0 HOPSX_PAR_WGRAD_MIN_FLOP=2e10; do run $k "cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10"; done
