set -o pipefail
o=gpurun_out/${1:-r5_pairknobs}; mkdir -p $o; export TMPDIR=/tmp
run() { env $1 timeout -k 10 200 python benchmarks/run.py cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10 > $o/r.json 2> $o/err.log || { tail -20 $o/err.log; exit 1; }
  echo "[$1] $(python -c "import json; r=json.loads(open('$o/r.json').read().strip().splitlines()[-1]); print(r['value'], r['ms_per_step'])")"; }
for k in X=0 HOPSX_PAIR_CPW=6 HOPSX_PAIR_CPW=24 HOPSX_PAIR_CPW=48 HOPSX_DGRAD_UN=1 HOPSX_DGRAD_XCD=1 X=0 HOPSX_WGRAD_NFKW=4; do run $k; done
