#!/bin/bash
# GEMM planner A/B (env knobs, no rebuild): tile floor for non-split GEMMs, split-K tile and target.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B="timeout -k 10 200 python -u benchmarks/run.py"
: > gpurun_out/plan_ab.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_v2_gpu.py tests/test_bnstats_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py \
  > gpurun_out/plan_tests.log 2>&1 || exit 1
run() {  # label, env..., then benchmark args after --
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  local out
  out=$(env "${envs[@]}" $B "$@" | tail -1 | cut -c1-150) || return 1
  echo "$label $* :: $out" >> gpurun_out/plan_ab.txt
}
run ks5off HOPSX_DISABLE=ks5 -- cifar_resnet --steps 20 --warmup 5 || exit 1
for cfg in cifar_resnet "resnet50 --batch 64" "resnet50 --batch 8"; do
  run default X=0 -- $cfg --steps 20 --warmup 5 && \
  run t64min256 HOPSX_GEMM_T64_MIN=256 -- $cfg --steps 20 --warmup 5 && \
  run splitcfg0 HOPSX_GEMM_SPLIT_CFG=0 -- $cfg --steps 20 --warmup 5 && \
  run splittgt4 HOPSX_GEMM_SPLIT_TARGET=4 -- $cfg --steps 20 --warmup 5 && \
  run splittgt1 HOPSX_GEMM_SPLIT_TARGET=1 -- $cfg --steps 20 --warmup 5 || exit 1
done
