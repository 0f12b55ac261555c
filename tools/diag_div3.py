"""Bench-divergence bisection: bench-identical loop with switches.
args: B graph record dist_init steps"""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
B = int(sys.argv[1]); graph = sys.argv[2] == "1"; record = sys.argv[3] == "1"; dinit = sys.argv[4] == "1"
steps = int(sys.argv[5])
if dinit:
    from hops_examples_amd.parallel import dist as hdist
    hdist.init()
from hops_examples_amd import optim
from hops_examples_amd.models.mnist import MirroredMnistCNN
from hops_examples_amd.runtime.arena import ParamArena
from hops_examples_amd.runtime.step import TrainStep
torch.manual_seed(1234)
dev = torch.device("cuda", 0)
m = MirroredMnistCNN().to(dev); ParamArena.from_module(m, dev)
opt = optim.Adadelta(m, lr=1.0)
st = TrainStep(m, opt, graph=graph)
nb = max(8, -(-61440 // B))
xs = torch.randint(0, 256, (nb, B, 28, 28, 1), dtype=torch.uint8, device=dev)
ys = torch.randint(0, 10, (nb, B), dtype=torch.int64, device=dev)
rec = torch.zeros(steps, device=dev)
chk = {}
for i in range(steps):
    r = st(xs[i % nb], ys[i % nb])
    if record:
        rec[i] = r["loss"].reshape(-1)[0]
    if i in (25, 50, 100, 150, 200, steps - 1):
        torch.cuda.synchronize()
        chk[i] = round(float(r["loss"].reshape(-1)[0]), 4)
        chk[f"w{i}"] = round(float(m._hx_arena.master.abs().max()), 3)
torch.cuda.synchronize()
print(json.dumps({"B": B, "graph": graph, "record": record, "dist_init": dinit, "chk": chk}), flush=True)
