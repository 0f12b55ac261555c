# data-parallel v2 taxi step on W = 2, 4, 8 processes sharing one GPU: steps/s, phase stamps; one-GPU phases
set -o pipefail
tag=${1:-taxidp}  # output under gpurun_out/<tag>/ (tools/gpu.sh taxidp <tag>)
mkdir -p gpurun_out/$tag
for w in 2 4 8; do
  mkdir -p gpurun_out/$tag/w$w
  timeout -k 10 200 python -c "
import sys; sys.path.insert(0,'.')
from hops_examples_amd.parallel import launch
sys.exit(launch.launch($w, ['tools/taxi_dp_worker.py','--out','gpurun_out/$tag/w$w','--steps','4','--bench','4000','--phases'], rehearse=True, timeout_s=180, extra_env={'HOPSX_TAXI_DP_TIMEOUT_S':'20'}))
" > gpurun_out/$tag/w$w/log.txt 2>&1 || exit 1
  cat gpurun_out/$tag/w$w/bench.json; echo; cat gpurun_out/$tag/w$w/phases.txt
done
timeout -k 10 120 python tools/taxi_phases.py 32 > gpurun_out/$tag/single_phases.txt 2>&1 && head -12 gpurun_out/$tag/single_phases.txt
