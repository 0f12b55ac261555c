set -o pipefail
o=gpurun_out/${1:-r5_e1ab}; mkdir -p $o; export TMPDIR=/tmp
for k in X=0 HOPSX_SMALLK_ITEMS=16 HOPSX_SMALLK_ITEMS=2; do
env $k timeout -k 10 300 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_keras_persist_gpu.py -k e1 > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
echo "[$k] $(grep "images/s" $o/t.log | cut -c1-160)"
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_conv_in_pool_gpu.py > $o/t2.log 2>&1 || { grep -E "FAIL|assert" $o/t2.log | tail -10; exit 1; }
tail -1 $o/t2.log
