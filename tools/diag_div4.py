"""Repeated graph-vs-eager runs in one process: find whether/when graph training explodes
and which parameter blows up first.  args: reps steps B [mode: graph|eager]"""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hops_examples_amd import optim
from hops_examples_amd.models.mnist import MirroredMnistCNN
from hops_examples_amd.runtime.arena import ParamArena
from hops_examples_amd.runtime.step import TrainStep
reps, steps, B = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
mode = sys.argv[4] if len(sys.argv) > 4 else "graph"
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
nb = max(8, -(-61440 // B))
g = torch.Generator(device=dev).manual_seed(7)
xs = torch.randint(0, 256, (nb, B, 28, 28, 1), dtype=torch.uint8, device=dev, generator=g)
ys = torch.randint(0, 10, (nb, B), dtype=torch.int64, device=dev, generator=g)
for rep in range(reps):
    torch.manual_seed(1234)
    m = MirroredMnistCNN().to(dev); ParamArena.from_module(m, dev)
    names = [n for n, _ in m.named_parameters()]
    opt = optim.Adadelta(m, lr=1.0)
    st = TrainStep(m, opt, graph=(mode == "graph"))
    bad = None
    t0 = time.time()
    for i in range(steps):
        st(xs[i % nb], ys[i % nb])
        if i % 5 == 4:
            torch.cuda.synchronize()
            mx = [p.detach().abs().max().item() for p in m.parameters()]
            if max(mx) > 2.0 or any(v != v for v in mx):
                bad = {"step": i, "maxabs": {n: round(v, 3) for n, v in zip(names, mx)}}
                break
    torch.cuda.synchronize()
    print(json.dumps({"rep": rep, "mode": mode, "B": B, "bad": bad, "s": round(time.time() - t0, 2)}), flush=True)
    del st, opt, m
