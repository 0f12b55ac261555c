#!/bin/bash
# gg engine weight-gradient A/B: default, main loop only (HOPSX_GG_DIAG=1), split caps.
# usage (through gpurun, repo root): tools/gpu_gg_ab.sh <tag> [batch]
set -o pipefail
tag=${1:-gg}; B=${2:-64}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 100 python tools/bench_wgrad.py --batch $B --glds-only > $out/default.jsonl 2>&1 || exit $?
HOPSX_GG_DIAG=1 timeout -k 10 100 python tools/bench_wgrad.py --batch $B --glds-only > $out/diag.jsonl 2>&1 || exit $?
HOPSX_GG_SPLIT_MAX=2 timeout -k 10 100 python tools/bench_wgrad.py --batch $B --glds-only > $out/smax2.jsonl 2>&1 || exit $?
HOPSX_GG_SPLIT_MAX=1 timeout -k 10 100 python tools/bench_wgrad.py --batch $B --glds-only > $out/smax1.jsonl 2>&1 || exit $?
HOPSX_GG_SPLIT_MAX=1 HOPSX_GG_DIAG=1 timeout -k 10 100 python tools/bench_wgrad.py --batch $B --glds-only > $out/smax1_diag.jsonl 2>&1 || exit $?
python tools/gg_ab_table.py $out
