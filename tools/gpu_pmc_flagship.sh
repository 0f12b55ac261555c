#!/bin/bash
# PMC passes over a short flagship run (bench.py MNIST only): instruction mix / MFMA / LDS conflicts,
# then HBM fetch and write bytes (one counter group per run, each under its own kill timer).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
P="python3 $R/bench.py --steps 40 --warmup 10 --no-taxi"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES -d "$R/gpurun_out/pmcf_a" -o run --output-format csv -- $P > "$R/gpurun_out/pmcf_a.log" 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES FETCH_SIZE -d "$R/gpurun_out/pmcf_b" -o run --output-format csv -- $P > "$R/gpurun_out/pmcf_b.log" 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES WRITE_SIZE -d "$R/gpurun_out/pmcf_c" -o run --output-format csv -- $P > "$R/gpurun_out/pmcf_c.log" 2>&1
rc=$?
find $R/gpurun_out/pmcf_a $R/gpurun_out/pmcf_b $R/gpurun_out/pmcf_c -name '*counter_collection.csv' | head
exit $rc
