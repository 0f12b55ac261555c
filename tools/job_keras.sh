set -o pipefail
o=gpurun_out/${1:-r5_keras}; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_keras_persist_gpu.py $(grep -ln "keras" tests/*_gpu.py | grep -v test_keras_persist_gpu | tr '\n' ' ') > $o/t.log 2>&1 || { grep -E "PASS|FAIL|Error|error|assert|images/s" $o/t.log | tail -30; exit 1; }
grep -E "images/s|passed|failed" $o/t.log | tail -4
