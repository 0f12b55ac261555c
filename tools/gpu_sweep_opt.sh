# optimizer store-policy A/B on the flagship bench (one GPU); base first and last for noise
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python -u bench.py --no-taxi --steps 1000 --warmup 20 > gpurun_out/sweep_base.log 2>&1 || exit 1
HOPSX_OPT_NT=1 timeout -k 10 120 python -u bench.py --no-taxi --steps 1000 --warmup 20 > gpurun_out/sweep_nt1.log 2>&1 || exit 1
HOPSX_OPT_NT=1 HOPSX_OPT_GRID=512 timeout -k 10 120 python -u bench.py --no-taxi --steps 1000 --warmup 20 \
  > gpurun_out/sweep_nt1_grid512.log 2>&1 || exit 1
timeout -k 10 120 python -u bench.py --no-taxi --steps 1000 --warmup 20 > gpurun_out/sweep_base2.log 2>&1
