set -o pipefail
o=gpurun_out/${1:-r5_ts}; mkdir -p $o; export TMPDIR=/tmp
HOPSX_PERSIST=0 timeout -k 10 200 rocprofv3 --kernel-trace -d $o/pf -o run -- python3 bench.py --steps 64 --warmup 10 --no-taxi > $o/b.log 2>&1 || { tail -20 $o/b.log; exit 1; }
db=$(find $o/pf -name '*.db' | head -1); python tools/step_kernels.py "$db" "void optim_k" > $o/step.txt 2>&1; rm -rf $o/pf
cat $o/step.txt | cut -c1-130
