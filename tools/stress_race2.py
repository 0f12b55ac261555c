"""Why do graph replays drift?  Variants (arg): alloc | noalloc | poison.  Also checks that
weights (master/shadow) and the input stay bit-identical across replays (out-of-bounds writes)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hops_examples_amd.models.mnist import MirroredMnistCNN
from hops_examples_amd.ops import functional as HF
from hops_examples_amd.runtime.arena import ParamArena
variant, N, B = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
dev = torch.device("cuda", 0)
torch.manual_seed(1234)
m = MirroredMnistCNN().to(dev); ParamArena.from_module(m, dev)
a = m._hx_arena
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
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    fb()
a.grad.zero_(); g.replay(); torch.cuda.synchronize()
ref, oref = a.grad.clone(), box["out"].detach().float().clone()
m0, s0, x0 = a.master.clone(), a.shadow.clone(), x.clone()
dbuf = torch.empty_like(ref); dmax = torch.zeros(N, device=dev); omax = torch.zeros(N, device=dev)
obuf = torch.empty_like(oref)
for i in range(N):
    a.grad.zero_()
    g.replay()
    if variant == "noalloc":
        torch.sub(a.grad, ref, out=dbuf); dbuf.abs_()
        torch.amax(dbuf, dim=0, out=dmax[i])
        obuf.copy_(box["out"].detach()); obuf.sub_(oref).abs_()
        torch.amax(obuf.view(-1), dim=0, out=omax[i])
    else:
        dmax[i] = (a.grad - ref).abs().max()
        omax[i] = (box["out"].detach().float() - oref).abs().max()
        if variant == "poison":
            p = torch.full((16 << 20,), float("nan"), device=dev)
            del p
torch.cuda.synchronize()
res = {"variant": variant, "N": N, "B": B,
       "grad_dev_max": float(dmax.max()), "first_grad_bad": int((dmax > 1e-3 * ref.abs().max()).nonzero()[0]) if (dmax > 1e-3 * ref.abs().max()).any() else None,
       "logit_dev_max": float(omax.max()),
       "master_changed": bool((a.master != m0).any()), "shadow_changed": bool((a.shadow != s0).any()),
       "input_changed": bool((x != x0).any())}
print(json.dumps(res), flush=True)
