set -o pipefail
o=gpurun_out/r5_rh; mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_bnstats_gpu.py -k "fp64 or matches_unfused" > $o/bn64.log 2>&1; tail -5 $o/bn64.log; grep "fp64 cos" $o/bn64.log
for cfg in "5 2" "64 10"; do set -- $cfg
  HOPSX_RANK_FAST_EXIT=0 timeout -k 10 240 python -u bench.py --gpus 2 --rehearse --steps $1 --warmup $2 --no-taxi > $o/rh_$1.json 2> $o/rh_$1.err || exit 1
  tail -1 $o/rh_$1.json | cut -c1-330
done
T=240 tools/rehearse_prof.sh $o/prof 2 bench.py --gpus 2 --rehearse --steps 5 --warmup 2 --no-taxi || { tail -20 $o/prof/r0.log; exit 1; }
tail -1 $o/prof/r0.log | cut -c1-300
python tools/rank_timeline.py $o/prof 2 "" 80 > $o/timeline.txt 2>&1; head -30 $o/timeline.txt
