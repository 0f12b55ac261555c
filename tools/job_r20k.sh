set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_stem_pad_gpu.py tests/test_models_gpu.py tests/test_bnstats_gpu.py > gpurun_out/${1:-r5_r20k}_tests.log 2>&1; tail -3 gpurun_out/${1:-r5_r20k}_tests.log
o=gpurun_out/${1:-r5_r20k}; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $o/pf -o run -- python3 benchmarks/run.py cifar_resnet --depth 20 --batch 128 --steps 20 --warmup 10 --inline > $o/pf.log 2>&1 || { tail -20 $o/pf.log; exit 1; }
db=$(find $o/pf -name '*.db' | head -1); python tools/step_kernels.py "$db" > $o/r20_step.txt 2>&1; rm -rf $o/pf
grep -n "non-hopsx\|one step" $o/r20_step.txt | head -40
timeout -k 10 300 rocprofv3 --kernel-trace -d $o/pf5 -o run -- python3 benchmarks/run.py resnet50 --batch 64 --steps 8 --warmup 5 > $o/pf5.log 2>&1 || { tail -20 $o/pf5.log; exit 1; }
db=$(find $o/pf5 -name '*.db' | head -1); python tools/step_kernels.py "$db" > $o/r50_step.txt 2>&1; rm -rf $o/pf5
grep -n "non-hopsx\|one step" $o/r50_step.txt | head -40
bash tools/gpu.sh ab ${1:-r5_r20k}_ab 1 "cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10" "HOPSX_DISABLE=pad_cin"
bash tools/gpu.sh ab ${1:-r5_r20k}_ab50 1 "resnet50 --batch 8 --steps 30 --warmup 5" "HOPSX_DISABLE=pad_cin"
