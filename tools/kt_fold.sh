set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/kt
for v in fold nofold; do
  if [ $v = nofold ]; then export HOPSX_DISABLE=bn_fold; else export HOPSX_DISABLE=; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/kt/$v -o run -- python3 benchmarks/run.py cifar_resnet --depth 20 --batch 128 --steps 30 --warmup 5 --inline > gpurun_out/kt/$v.log 2>&1 || exit 1
  db=$(find gpurun_out/kt/$v -name '*.db' | head -1); python tools/profdb.py "$db" > gpurun_out/kt/$v.txt 2>&1
  rm -rf gpurun_out/kt/$v
done
