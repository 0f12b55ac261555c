set -o pipefail
o=gpurun_out/${1:-r5_e1prof}; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/pf -o run -- python3 tools/e1_fit.py > $o/pf.log 2>&1 || { tail -20 $o/pf.log; exit 1; }
db=$(find $o/pf -name '*.db' | head -1); python tools/profdb.py "$db" > $o/e1_kernels.txt 2>&1; python tools/step_kernels.py "$db" "void optim_k" > $o/e1_step.txt 2>&1; rm -rf $o/pf
head -22 $o/e1_kernels.txt | cut -c1-140; head -30 $o/e1_step.txt | cut -c1-120
