"""Optimizer kernel timing at the MNIST arena size (1.39 M params), Adadelta, with/without the
arrival counter (step/RNG bump by the last workgroup)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hops_examples_amd.ops import kernels as K
dev = torch.device("cuda", 0)
n = 1394368
p = torch.randn(n, device=dev); g = torch.randn(n, device=dev) * 1e-3
s1 = torch.zeros(n, device=dev); s2 = torch.zeros(n, device=dev)
sh = torch.empty(n, device=dev, dtype=torch.bfloat16)
step = torch.zeros(1, device=dev); arr = torch.zeros(1, device=dev, dtype=torch.int32)
rng = torch.zeros(2, device=dev, dtype=torch.int64)
res = {}
for name, kw in (("arrive", dict(step_dev=step, arrive=arr, rng=rng)), ("noarrive", dict(step_dev=None))):
    f = lambda: K.optim_step(3, p, g, s1, s2, None, sh, [1.0, 1.0, 0.0, 0.95, 1e-7], zero_grad=True, **kw)
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(200):
        f()
    b.record()
    torch.cuda.synchronize()
    res[name] = round(a.elapsed_time(b) * 1000 / 200, 2)
print(json.dumps({"grid_cap": os.environ.get("HOPSX_OPT_GRID", "512"), "us": res}), flush=True)
