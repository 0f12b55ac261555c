"""Diagnose training divergence: loss trajectory on a large random pool with fast paths on/off."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hops_examples_amd import optim
from hops_examples_amd.models.mnist import MirroredMnistCNN
from hops_examples_amd.runtime.arena import ParamArena
from hops_examples_amd.runtime.step import TrainStep
B = int(sys.argv[1]); graph = sys.argv[2] == "1"; steps = int(sys.argv[3]) if len(sys.argv) > 3 else 400
torch.manual_seed(1234)
m = MirroredMnistCNN().cuda(); ParamArena.from_module(m)
opt = optim.Adadelta(m, lr=1.0)
st = TrainStep(m, opt, graph=graph)
nb = max(8, -(-61440 // B))
xs = torch.randint(0, 256, (nb, B, 28, 28, 1), dtype=torch.uint8, device="cuda")
ys = torch.randint(0, 10, (nb, B), device="cuda")
traj = []
first_bad = None
for i in range(steps):
    r = st(xs[i % nb], ys[i % nb])
    if i % 25 == 0 or first_bad is None:
        l = float(r["loss"].item())
        if i % 25 == 0:
            traj.append(round(l, 3))
        if first_bad is None and (l != l or l > 10):
            first_bad = i
            g = opt.arena.grad
            print(json.dumps({"first_bad_step": i, "loss": l, "wmax": float(opt.arena.master.abs().max()),
                              "s1max": float(opt._states[0].abs().max()), "s2max": float(opt._states[1].abs().max())}))
print(json.dumps({"B": B, "graph": graph, "disable": os.environ.get("HOPSX_DISABLE", ""), "traj": traj,
                  "wmax": float(opt.arena.master.abs().max())}))
