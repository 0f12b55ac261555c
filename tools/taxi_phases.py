"""Phase timestamps of the fused taxi step kernel (HOPSX_PHASE_DBG=1)."""
import os, sys
os.environ["HOPSX_PHASE_DBG"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hops_examples_amd.models import widedeep as WD
from hops_examples_amd.runtime.arena import ParamArena

dev = torch.device("cuda", 0)
B, nb = 40, 16
dense, cat, label = WD.synth_taxi(nb * B, seed=3, device=dev)
m = WD.TaxiWideDeep().to(dev)
ParamArena.from_module(m, dev)
fs = WD.FusedWideDeepStep(m, WD.make_optimizer(m))
xs, ys = (dense.view(nb, B, -1), cat.view(nb, B, -1)), label.view(nb, B, 1)
names = {0: "start", 1: "staged", 10: "loss"}
names.update({2 + l: f"fwd{l}" for l in range(8)})
names.update({11 + l: f"bwd{l}" for l in range(8)})
names[19] = "end"
acc = {}
for it in range(30):
    fs.step_resident(xs, ys, graph=False)
    torch.cuda.synchronize()
    t = fs.dbg.cpu().tolist()
    if it >= 10:
        for k in range(1, 20):
            if t[k] and t[0]:
                acc.setdefault(k, []).append((t[k] - t[0]) / 100.0)
for k in sorted(acc):
    v = acc[k]
    print(f"{names[k]:8s} t+{sum(v) / len(v):7.2f} us")
