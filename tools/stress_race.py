"""Race hunt: replay fwd+bwd (no optimizer) on FIXED weights/inputs thousands of times and compare
every replay's gradients / logits with the first one.  Deterministic kernels must match bit-for-bit;
atomic-accumulating ones to fp32 rounding.  args: N B mode(graph|eager)"""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hops_examples_amd.models.mnist import MirroredMnistCNN
from hops_examples_amd.ops import functional as HF
from hops_examples_amd.runtime.arena import ParamArena
N, B, mode = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
dev = torch.device("cuda", 0)
torch.manual_seed(1234)
m = MirroredMnistCNN().to(dev); ParamArena.from_module(m, dev)
a = m._hx_arena
names = [n for n, _ in m.named_parameters()]
ranges = [(o, o + p.numel()) for p, o in zip(a.params, a.offsets)]
x = torch.randint(0, 256, (B, 28, 28, 1), dtype=torch.uint8, device=dev)
y = torch.randint(0, 10, (B,), device=dev)
box = {}
def fb():
    out = m(x)
    loss, corr, cnt, dl = HF.loss_and_grad(out, y, "sparse_ce")
    out.backward(dl)
    box["out"] = out
for _ in range(3):
    fb(); a.grad.zero_()
torch.cuda.synchronize()
if mode == "graph":
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fb()
    run = g.replay
else:
    run = fb
a.grad.zero_(); run(); torch.cuda.synchronize()
ref = a.grad.clone(); oref = box["out"].float().clone()
scale = torch.stack([ref[s:e].abs().max() for s, e in ranges]) + 1e-12
rec = torch.zeros(N, len(ranges) + 1, device=dev)
for i in range(N):
    a.grad.zero_()
    run()
    d = (a.grad - ref).abs()
    rec[i, :-1] = torch.stack([d[s:e].max() for s, e in ranges]) / scale
    rec[i, -1] = (box["out"].float() - oref).abs().max() / (oref.abs().max() + 1e-12)
torch.cuda.synchronize()
mx = rec.max(0).values.tolist()
bad = (rec > 1e-2).any(1).nonzero().flatten().tolist()
print(json.dumps({"mode": mode, "N": N, "B": B, "disable": os.environ.get("HOPSX_DISABLE", ""),
                  "max_rel_dev": {n: float(f"{v:.3g}") for n, v in zip(names + ["logits"], mx)},
                  "n_bad": len(bad), "first_bad": bad[:10],
                  "bad_rows": [[float(f"{v:.3g}") for v in rec[i].tolist()] for i in bad[:5]]}), flush=True)
