# round-5 zero-copy / overlapped DP checks on one GPU (2 ranks sharing it)
set -o pipefail
o=gpurun_out/r5_dp; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_p2p_gpu.py tests/test_oneshot_gpu.py > $o/p2p.log 2>&1; rc=$?; tail -12 $o/p2p.log; grep DPFUSED $o/p2p.log | cut -c1-700
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for m in overlap copy; do
  if [ $m = copy ]; then export HOPSX_P2P_ZEROCOPY=0; fi
  T=400 tools/rehearse_prof.sh $o/r50_$m 2 benchmarks/run.py resnet50 --gpus 2 --rehearse --batch 32 --steps 6 --warmup 5 || { tail -30 $o/r50_$m/r0.log; exit 1; }
  grep images/sec $o/r50_$m/r0.log | cut -c1-600
  python tools/rank_timeline.py $o/r50_$m 2 "" 120 > $o/r50_$m/timeline.txt 2>&1
  python tools/profdb.py $o/r50_$m/r0.db "r50 2 ranks $m rank0" > $o/r50_$m/k0.txt 2>&1; head -14 $o/r50_$m/k0.txt
  python tools/rank_timeline.py $o/r50_$m 2 dp_step_k 400 > $o/r50_$m/timeline_step.txt 2>&1
  rm -f $o/r50_$m/*.db   # (the traces are >64 MiB: only the summaries travel back)
done
