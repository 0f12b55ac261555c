#!/bin/bash
# PMC passes over a short ResNet-20 run (one counter group per run, each under its own kill timer):
# instruction mix / MFMA / LDS conflicts, then HBM fetch and write bytes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
P="python3 $R/benchmarks/run.py cifar_resnet --steps 4 --warmup 3"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES -d "$R/gpurun_out/pmc_a" -o run --output-format csv -- $P > "$R/gpurun_out/pmc_a.log" 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES FETCH_SIZE -d "$R/gpurun_out/pmc_b" -o run --output-format csv -- $P > "$R/gpurun_out/pmc_b.log" 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES WRITE_SIZE -d "$R/gpurun_out/pmc_c" -o run --output-format csv -- $P > "$R/gpurun_out/pmc_c.log" 2>&1
