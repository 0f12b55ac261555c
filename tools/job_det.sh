set -o pipefail
o=gpurun_out/${1:-r5_det}; mkdir -p $o; export TMPDIR=/tmp
HOPSX_DETERMINISTIC=1 timeout -k 10 200 python tools/det_diag.py > $o/diag.txt 2>&1 || { tail -20 $o/diag.txt; exit 1; }
tail -1 $o/diag.txt
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_deterministic_gpu.py tests/test_bn_dgrad_sums_gpu.py tests/test_bnstats_gpu.py tests/test_keras_persist_gpu.py > $o/t.log 2>&1 || { grep -E "FAIL|Error|assert" $o/t.log | tail -20; exit 1; }
tail -1 $o/t.log
timeout -k 10 200 python benchmarks/run.py cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10 2>/dev/null | tail -1 | cut -c1-200
