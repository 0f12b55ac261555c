#!/bin/bash
# kernel trace + two counter passes over tools/mb_conv.py (one block-limited pass per run)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 -u "$R/tools/mb_conv.py" > "$R/gpurun_out/pmc_mb.log" 2>&1 && \
timeout -k 10 120 python3 -u "$R/tools/dbg_convfwd.py" > "$R/gpurun_out/dbg_convfwd.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/pmc_conv_t" -o run --output-format csv -- python3 "$R/tools/mb_conv.py" > "$R/gpurun_out/pmc_t.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d "$R/gpurun_out/pmc_conv1" -o run --output-format csv -- python3 "$R/tools/mb_conv.py" > "$R/gpurun_out/pmc_1.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_MFMA -d "$R/gpurun_out/pmc_conv2" -o run --output-format csv -- python3 "$R/tools/mb_conv.py" > "$R/gpurun_out/pmc_2.log" 2>&1
