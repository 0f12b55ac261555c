#!/bin/bash
# Multi-rank rehearsal on ONE GPU with a rocprofv3 kernel trace per rank (no launcher process: each
# rank is started here under its own profiler, so nothing execs from a process that touched the GPU).
#   tools/rehearse_prof.sh <outdir> <nranks> <script + args...>
# -> <outdir>/r<k>.db (+ _kernel_stats.csv, .log) for every rank; tools/profdb.py / tools/rank_timeline.py read them
set -o pipefail
out=${1:?outdir}; n=${2:?nranks}; shift 2
mkdir -p $out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 HOPSX_DIST_BACKEND=gloo PYTHONUNBUFFERED=1
port=$((29500 + RANDOM % 2000))
pids=()
for ((r = 0; r < n; r++)); do
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=$n LOCAL_WORLD_SIZE=$n GROUP_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port \
    timeout -k 10 ${T:-300} rocprofv3 --kernel-trace --stats -d $out/p$r -o run -- python3 "$@" > $out/r$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
for ((r = 0; r < n; r++)); do
  db=$(find $out/p$r -name '*.db' | head -1); [ -n "$db" ] && cp "$db" $out/r$r.db
  f=$(find $out/p$r -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $out/r${r}_kernel_stats.csv
  rm -rf $out/p$r
done
exit $rc
