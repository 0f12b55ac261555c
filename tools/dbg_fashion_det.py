"""Which change moves the FashionMnistCNN logits: fused conv+pool (UN 1 / 2) vs unfused, repeated runs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from hops_examples_amd.models import mnist
from hops_examples_amd.ops import functional as HF
from hops_examples_amd.runtime.arena import ParamArena

dev = torch.device("cuda", 0)


def run(disable, un):
    os.environ["HOPSX_DISABLE"] = disable
    HF.seed_device_rng(9, dev)
    torch.manual_seed(0)
    m = mnist.FashionMnistCNN().to(dev)
    for mod in m.modules():
        if hasattr(mod, "salt"):
            mod.salt = 7919
    ParamArena.from_module(m, dev)
    x = torch.randint(0, 256, (32, 28, 28, 1), dtype=torch.uint8, device=dev)
    pooled = {}
    h = m.conv1(m.prep(x))
    out = m(x)
    torch.cuda.synchronize()
    return out.float().clone(), h.float().clone()


ref, h0 = run("conv_pool", 0)
for name, dis in [("unfused again", "conv_pool"), ("fused", "")]:
    o, h = run(dis, 0)
    print(name, "logits max|diff|", (o - ref).abs().max().item(), "n", int((o != ref).sum()), "conv1 diff",
          (h - h0).abs().max().item(), flush=True)
