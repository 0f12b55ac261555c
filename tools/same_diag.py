import torch, sys, os
sys.path.insert(0, os.getcwd())
from hops_examples_amd.ops import functional as HF
for k, C in ((2, 1), (3, 1), (2, 32)):
    x = torch.randn(4, 28, 28, C, device="cuda").to(torch.bfloat16).requires_grad_(True)
    w = torch.randn(32, k, k, C, device="cuda").requires_grad_(True); b = torch.randn(32, device="cuda").requires_grad_(True)
    y = HF.conv2d(x, w, b, padding="same", act="relu"); y.backward(torch.randn_like(y))
    print(k, C, tuple(y.shape), x.grad is None, w.grad is None, b.grad is None, flush=True)
