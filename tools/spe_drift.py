"""Pairwise weight-update distances: steps_per_execution graph vs one-step replays (and repeats)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hops_examples_amd import optim
from hops_examples_amd.models.mnist import MirroredMnistCNN
from hops_examples_amd.ops import functional as HF
from hops_examples_amd.runtime.arena import ParamArena
from hops_examples_amd.runtime.step import TrainStep

dev = torch.device("cuda", 0)
B, nb = 32, 6
n = int(sys.argv[1]) if len(sys.argv) > 1 else 23
g = torch.Generator().manual_seed(0)
xs = torch.randint(0, 256, (nb, B, 28, 28, 1), dtype=torch.uint8, generator=g).to(dev)
ys = torch.randint(0, 10, (nb, B), generator=g).to(dev)
res = {}
for tag, multi, drop in [("multi", True, True), ("multi2", True, True), ("single", False, True), ("single2", False, True),
                         ("multi_nodrop", True, False), ("single_nodrop", False, False)]:
    HF.seed_device_rng(11, dev)
    torch.manual_seed(0)
    m = MirroredMnistCNN().to(dev)
    m.pool.salt = 7919
    if not drop:
        m.pool.dropout = 0.0
    ParamArena.from_module(m, dev)
    w0 = m._hx_arena.master.clone()
    st = TrainStep(m, optim.SGD(m, lr=0.05), "sparse_ce", steps_per_execution=8)
    if multi:
        r = st.run_resident(xs, ys, n)
    else:
        for _ in range(n):
            r = st.step_resident(xs, ys)
    torch.cuda.synchronize()
    res[tag] = (m._hx_arena.master - w0).clone()
    print(tag, float(r["loss"].reshape(-1)[0]), int(st._cursor.item()))
for a, b in [("multi", "multi2"), ("single", "single2"), ("multi", "single"), ("multi_nodrop", "single_nodrop")]:
    d = float((res[a] - res[b]).norm()) / float(res[b].norm())
    print(f"{a:14s} vs {b:14s} rel {d:.4g}")
