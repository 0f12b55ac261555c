# one PMC pass over the flagship step: L2->memory fetch bytes and waves per kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE SQ_WAVES --output-format csv -d gpurun_out/pmc -o pmc -- \
  python3 bench.py --no-taxi --steps 40 --warmup 10 > gpurun_out/pmc.log 2>&1
