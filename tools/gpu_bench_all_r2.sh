# every BASELINE config through benchmarks/run.py on one MI355X (one JSON line each)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
B=gpurun_out/r2_benchmarks.log
: > $B
for c in "taxi" "titanic" "cifar_resnet --steps 50 --warmup 10" "cifar_resnet --depth 56 --steps 30 --warmup 5" \
         "resnet50 --steps 20 --warmup 5" "resnet50 --batch 64 --steps 20 --warmup 5" \
         "mnist_mirrored --batch 2048 --steps 100 --warmup 10"; do
  echo "== $c" >> $B
  timeout -k 10 240 python -u benchmarks/run.py $c >> $B 2>&1 || { echo "FAIL rc=$? $c" >> $B; exit 1; }
done
