set -o pipefail
o=gpurun_out/${1:-r5_b8knobs2}; mkdir -p $o; export TMPDIR=/tmp
run() { env $1 timeout -k 10 200 python benchmarks/run.py $2 > $o/r.json 2> $o/err.log || { tail -20 $o/err.log; exit 1; }
  echo "[$1] $2 -> $(python -c "import json; r=json.loads(open('$o/r.json').read().strip().splitlines()[-1]); print(r['value'], r['ms_per_step'])")"; }
for k in X=0 HOPSX_GG_MIN_WG=32 HOPSX_GEMM_SPLIT_TARGET=4 "HOPSX_GG_MIN_WG=32 HOPSX_GEMM_SPLIT_TARGET=4" X=0 "HOPSX_GG_MIN_WG=32 HOPSX_GEMM_SPLIT_TARGET=4"; do run "$k" "resnet50 --batch 8 --steps 30 --warmup 5"; done
for k in X=0 "HOPSX_GG_MIN_WG=32 HOPSX_GEMM_SPLIT_TARGET=4"; do run "$k" "resnet50 --batch 64 --steps 12 --warmup 4"; run "$k" "cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10"; done
