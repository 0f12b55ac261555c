set -o pipefail
o=gpurun_out/${1:-r5_b8table}; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/pf -o run -- python3 benchmarks/run.py resnet50 --batch 8 --steps 20 --warmup 5 > $o/pf.log 2>&1 || { tail -20 $o/pf.log; exit 1; }
db=$(find $o/pf -name '*.db' | head -1); python tools/profdb.py "$db" > $o/r50_b8_kernels.txt 2>&1; python tools/step_kernels.py "$db" > $o/r50_b8_step.txt 2>&1; rm -rf $o/pf
head -40 $o/r50_b8_kernels.txt | cut -c1-150; grep "one step" $o/r50_b8_step.txt
