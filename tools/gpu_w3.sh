cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp
for N in 2 4; do for V in 1 2 3; do
  HOPSX_WGRAD_NFKW=$N HOPSX_WGRAD_CPW=$V MB_ONLY=conv2_wgrad timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/w3_${N}_$V" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/microbench.py" 32 200 > /dev/null 2>&1 || exit 1
  echo "nfkw=$N cpw=$V $(python3 $GRAFT_REPO_ROOT/tools/profsum.py $GRAFT_REPO_ROOT/gpurun_out/w3_${N}_$V/run_kernel_stats.csv 1 1 | tail -1)" >> $GRAFT_REPO_ROOT/gpurun_out/w3.txt
done; done
