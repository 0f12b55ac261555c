"""Diagnose training divergence at B=256: loss trajectory with fast paths on/off."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hops_examples_amd import optim
from hops_examples_amd.models.mnist import MirroredMnistCNN
from hops_examples_amd.runtime.arena import ParamArena
from hops_examples_amd.runtime.step import TrainStep
B = int(sys.argv[1]); graph = sys.argv[2] == "1"
torch.manual_seed(1234)
m = MirroredMnistCNN().cuda(); ParamArena.from_module(m)
opt = optim.Adadelta(m, lr=1.0)
st = TrainStep(m, opt, graph=graph)
xs = torch.randint(0, 256, (8, B, 28, 28, 1), dtype=torch.uint8, device="cuda")
ys = torch.randint(0, 10, (8, B), device="cuda")
traj = []
for i in range(240):
    r = st(xs[i % 8], ys[i % 8])
    if i % 20 == 0:
        traj.append(round(float(r["loss"].item()), 4))
print(json.dumps({"B": B, "graph": graph, "disable": os.environ.get("HOPSX_DISABLE", ""), "traj": traj,
                  "wmax": float(opt.arena.master.abs().max().item())}))
