set -o pipefail
o=gpurun_out/${1:-r5_b8knobs}; mkdir -p $o; export TMPDIR=/tmp
run() { env $1 timeout -k 10 200 python benchmarks/run.py resnet50 --batch 8 --steps 30 --warmup 5 > $o/r.json 2> $o/err.log || { tail -20 $o/err.log; exit 1; }
  echo "[$1] $(python -c "import json; r=json.loads(open('$o/r.json').read().strip().splitlines()[-1]); print(r['value'], r['ms_per_step'])")"; }
for k in X=0 HOPSX_GG_MIN_WG=32 HOPSX_GG_MIN_WG=16 HOPSX_CONV_SPLIT_MINK=1024 HOPSX_GG_SPLIT_TARGET=2 HOPSX_GEMM_SPLIT_TARGET=4 HOPSX_PAR_WGRAD_MIN_FLOP=1e8 HOPSX_PAR_WGRAD_MIN_FLOP=2e10 HOPSX_GG_MIN_N=33 X=0; do run $k; done
