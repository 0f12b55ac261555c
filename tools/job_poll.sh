# persistent flagship: multi-wave staggered polling knob (HOPSX_PERSIST_POLLW / _STAGGER)
set -o pipefail
o=gpurun_out/${1:-r5_poll}; mkdir -p $o; export TMPDIR=/tmp
HOPSX_PERSIST_CSTREAM=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_persist_gpu.py tests/test_persist_dp_gpu.py > $o/tests4.log 2>&1; rc=$?; tail -3 $o/tests4.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
for s in "HOPSX_PERSIST_POLLW_C=1" "" "HOPSX_PERSIST_CSTREAM=1" "HOPSX_PERSIST_POLLW_A=2" "HOPSX_PERSIST_POLLW_B=2" "HOPSX_PERSIST_POLLW_D=2" "HOPSX_PERSIST_CSTREAM=1 HOPSX_PERSIST_POLLW_D=2"; do
  r=$(env $s timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-taxi 2>>$o/err.log) || { echo "FAIL [$s]"; tail -20 $o/err.log; exit 1; }
  echo "[$s] $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a $o/ab.txt
done; done
for s in "HOPSX_PERSIST_CSTREAM=0" "HOPSX_PERSIST_CSTREAM=1"; do
  env $s timeout -k 10 240 python -u tools/persist_check.py --steps 8 --timing 32 > "$o/check_${s##*=}.log" 2>&1 || { tail -20 "$o/check_${s##*=}.log"; exit 1; }
  grep -A14 "host wall" "$o/check_${s##*=}.log"
done
