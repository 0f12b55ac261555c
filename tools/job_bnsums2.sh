set -o pipefail
o=gpurun_out/${1:-r5_bns2}; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $o/pf -o run -- python3 benchmarks/run.py cifar_resnet --depth 20 --batch 128 --steps 20 --warmup 10 --inline > $o/pf.log 2>&1 || { tail -20 $o/pf.log; exit 1; }
db=$(find $o/pf -name '*.db' | head -1); python tools/step_kernels.py "$db" > $o/r20_step.txt 2>&1; rm -rf $o/pf
grep -n "non-hopsx\|one step" $o/r20_step.txt | head
run() { env $1 timeout -k 10 300 python benchmarks/run.py $2 > $o/r.json 2> $o/err.log || { tail -20 $o/err.log; exit 1; }
  echo "[$1] $2 -> $(python -c "import json; r=json.loads(open('$o/r.json').read().strip().splitlines()[-1]); print(r['value'], r['ms_per_step'])")"; }
for d in X=0 HOPSX_DISABLE=bn_dgrad_sums; do
  run $d "cifar_resnet --depth 56 --batch 128 --steps 60 --warmup 10"
  run $d "resnet50 --batch 8 --steps 30 --warmup 5"
  run $d "resnet50 --batch 64 --steps 12 --warmup 4"
done
