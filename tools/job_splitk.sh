# conv split-K + RMSprop-lite: tests, per-layer table at B=8, ResNet-50 A/Bs
set -o pipefail
o=gpurun_out/${1:-r5_sk}; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_conv_splitk_gpu.py tests/test_kernels_gpu.py tests/test_bnstats_gpu.py > $o/tests.log 2>&1; rc=$?; tail -4 $o/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $o/tests.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/bench_conv_gemm.py --batch 8 --torch > $o/convgemm_b8.jsonl 2> $o/convgemm_b8.err || { tail -20 $o/convgemm_b8.err; exit 1; }
tail -1 $o/convgemm_b8.jsonl
bash tools/gpu.sh ab ${1:-r5_sk}_ab 2 "resnet50 --batch 8 --steps 30 --warmup 5" "HOPSX_DISABLE=conv_splitk"
bash tools/gpu.sh ab ${1:-r5_sk}_ab64 1 "resnet50 --batch 64 --steps 20 --warmup 5" "HOPSX_DISABLE=conv_splitk"
bash tools/gpu.sh ab ${1:-r5_sk}_ab256 1 "resnet50 --batch 256 --steps 10 --warmup 3"
bash tools/gpu.sh ab ${1:-r5_sk}_abc 1 "cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10"
