#!/bin/bash
# Kernel table of the ResNet-50 B=8 step (the reference benchmark notebook's config).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r50b8" -o run --output-format csv -- python3 "$R/benchmarks/run.py" resnet50 --batch 8 --steps 20 --warmup 5 > "$R/gpurun_out/prof_r50b8.log" 2>&1
