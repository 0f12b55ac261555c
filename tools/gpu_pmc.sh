#!/bin/bash
# PMC counter passes over selected microbench ops (one rocprofv3 run per counter group)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-pmc}
export MB_ONLY=${2:-conv2_dgrad,conv2_dgrad_fused}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_kt" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/microbench.py" 32 200 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_kt.log" 2>&1 || exit 1
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" "SQ_INSTS_MFMA SQ_WAIT_ANY SQ_INSTS_FLAT SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU" "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $C -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_p$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/microbench.py" 32 50 > "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_p$i.log" 2>&1 || exit 1
done
