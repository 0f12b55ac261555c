#!/bin/bash
# PMC passes over one gg weight-gradient layer (rocprofv3 --pmc, one pass per counter group).
# usage (through gpurun, repo root): tools/gpu_gg_pmc.sh <tag> <H,C,CO,k,s> [batch]
# A pass that fails for a counter name does not stop the others; a timeout / kill / abort /
# segfault ends the script (no further GPU work after it).
tag=${1:-pmc}; layer=${2:-7,512,512,3,1}; B=${3:-64}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $out/counters.txt 2>&1
rc=$?; case $rc in 124|137|134|139) exit $rc;; esac
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_VMEM TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $out/p$i -o run -- python3 tools/bench_wgrad.py --batch $B --glds-only --only $layer --iters 10 > $out/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc" >> $out/status.txt
  case $rc in 124|137|134|139) exit $rc;; esac
done
exit 0
