#!/bin/bash
# conv backward pair kernel vs fp32 (incl. the new KS=9 instantiation) + the model-level pair test.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_v2_gpu.py -k "bwd_pair_kernel or paired_conv" > gpurun_out/pair_tests.log 2>&1
rc=$?
exit $rc
