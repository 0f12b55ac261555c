set -o pipefail
o=gpurun_out/${1:-r5_pool}; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels_v2_gpu.py tests/test_conv_in_pool_gpu.py tests/test_models_gpu.py tests/test_persist_gpu.py > $o/t.log 2>&1 || { grep -E "FAIL|assert|Error" $o/t.log | tail -10; exit 1; }
tail -1 $o/t.log
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_keras_persist_gpu.py > $o/t2.log 2>&1 || { tail -20 $o/t2.log; exit 1; }
grep -E "images/s|passed" $o/t2.log | cut -c1-200
