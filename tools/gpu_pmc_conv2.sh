#!/bin/bash
# LDS / TLB / latency counter passes over tools/mb_conv.py
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH -d "$R/gpurun_out/pmc_c3" -o run --output-format csv -- python3 "$R/tools/mb_conv.py" > "$R/gpurun_out/pmc_3.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ -d "$R/gpurun_out/pmc_c4" -o run --output-format csv -- python3 "$R/tools/mb_conv.py" > "$R/gpurun_out/pmc_4.log" 2>&1
