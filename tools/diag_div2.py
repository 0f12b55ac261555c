"""Divergence vs host synchronisation: record per-step loss on device without syncing."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hops_examples_amd import optim
from hops_examples_amd.models.mnist import MirroredMnistCNN
from hops_examples_amd.runtime.arena import ParamArena
from hops_examples_amd.runtime.step import TrainStep
B = int(sys.argv[1]); graph = sys.argv[2] == "1"; steps = int(sys.argv[3]); sync = sys.argv[4] == "1"
torch.manual_seed(1234)
dev = torch.device("cuda", 0)
m = MirroredMnistCNN().to(dev); ParamArena.from_module(m, dev)
opt = optim.Adadelta(m, lr=1.0)
st = TrainStep(m, opt, graph=graph)
nb = max(8, -(-61440 // B))
xs = torch.randint(0, 256, (nb, B, 28, 28, 1), dtype=torch.uint8, device=dev)
ys = torch.randint(0, 10, (nb, B), device=dev)
rec = torch.zeros(steps, device=dev)
for i in range(steps):
    r = st(xs[i % nb], ys[i % nb])
    rec[i] = r["loss"][0] if r["loss"].dim() else r["loss"]
    if sync:
        torch.cuda.synchronize()
torch.cuda.synchronize()
l = rec.cpu().tolist()
bad = next((i for i, v in enumerate(l) if not (v == v) or v > 10), None)
print(json.dumps({"B": B, "graph": graph, "sync": sync, "disable": os.environ.get("HOPSX_DISABLE", ""),
                  "first_bad": bad, "traj": [round(v, 3) for v in l[::30]]}))
