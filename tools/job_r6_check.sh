# round-6 check: taxi DP phases + tests, ResNet per-layer numerics, the tightened whole-step tests
set -o pipefail
bash tools/taxi_dp_phases.sh || exit 1
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_taxi_dp_gpu.py tests/test_taxi_v2_gpu.py > gpurun_out/r6j/pytest.log 2>&1; tail -3 gpurun_out/r6j/pytest.log
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_resnet_layers_gpu.py tests/test_bnstats_gpu.py tests/test_kernels_v2_gpu.py tests/test_bn_dgrad_sums_gpu.py > gpurun_out/r6j/layers.log 2>&1; tail -5 gpurun_out/r6j/layers.log
timeout -k 10 400 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_p2p_gpu.py > gpurun_out/r6j/p2p.log 2>&1; tail -4 gpurun_out/r6j/p2p.log; grep DPRESNET gpurun_out/r6j/p2p.log | cut -c1-600
