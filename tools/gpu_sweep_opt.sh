# optimizer grid-cap sweep on the flagship bench (one GPU); base run first and last for noise
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python -u bench.py --no-taxi --steps 1000 --warmup 20 > gpurun_out/sweep_base.log 2>&1 || exit 1
for gcap in 128 192 256 320; do
  HOPSX_OPT_GRID=$gcap timeout -k 10 120 python -u bench.py --no-taxi --steps 1000 --warmup 20 \
    > gpurun_out/sweep_grid$gcap.log 2>&1 || exit 1
done
timeout -k 10 120 python -u bench.py --no-taxi --steps 1000 --warmup 20 > gpurun_out/sweep_base2.log 2>&1
