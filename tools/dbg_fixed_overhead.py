"""Fixed cost of a timed window of the flagship bench: wall time of run_resident(n) for several n
(linear fit -> per-step time + fixed overhead), and the host time of one graph replay call."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hops_examples_amd import optim
from hops_examples_amd.models.mnist import MirroredMnistCNN
from hops_examples_amd.runtime.arena import ParamArena
from hops_examples_amd.runtime.step import TrainStep
dev = torch.device("cuda", 0)
m = MirroredMnistCNN().to(dev); ParamArena.from_module(m, dev)
st = TrainStep(m, optim.Adadelta(m, lr=1.0), "sparse_ce")
nb, B = 1920, 32
xs = torch.randint(0, 256, (nb, B, 28, 28, 1), dtype=torch.uint8, device=dev)
ys = torch.randint(0, 10, (nb, B), device=dev)
for _ in range(5):
    st.step_resident(xs, ys)
res = {}
for n in (8, 16, 20, 24, 40, 200):
    st.prepare_resident(xs, ys, n=n)
    ts = []
    for rep in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st.run_resident(xs, ys, n)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ts.append((t2 - t0, t1 - t0))
    ts.sort()
    res[n] = {"wall_us": round(ts[2][0] * 1e6, 1), "host_issue_us": round(ts[2][1] * 1e6, 1)}
torch.cuda.synchronize()
t0 = time.perf_counter(); st._gU.replay(); t1 = time.perf_counter(); torch.cuda.synchronize(); t2 = time.perf_counter()
res["one_gU_replay"] = {"host_us": round((t1 - t0) * 1e6, 1), "wall_us": round((t2 - t0) * 1e6, 1)}
torch.cuda.synchronize()
t0 = time.perf_counter(); torch.cuda.synchronize(); res["empty_sync_us"] = round((time.perf_counter() - t0) * 1e6, 1)
print(json.dumps(res), flush=True)
