"""Time the flagship's conv kernels standalone (MNIST CNN at batch 32): conv2 fwd+pool, conv2
backward pair (dgrad with the input layer's wgrad fused + wgrad), conv1 direct forward.
Numerics are checked against the unfused chain first.  Usage: python tools/mb_conv.py [B]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from hops_examples_amd.ops import functional as HF
from hops_examples_amd.ops import kernels as K

dev = torch.device("cuda", 0)
bf = torch.bfloat16
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
torch.manual_seed(0)


def timeit(fn, n=300):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1000.0


x0 = torch.randint(0, 256, (B, 28, 28, 1), device=dev, dtype=torch.uint8)
w1 = (torch.randn(32, 2, 2, 1, device=dev) * 0.3).to(bf)
b1 = torch.randn(32, device=dev) * 0.1
g1 = K.conv_geom(x0.shape, w1.shape, (1, 1), (0, 0), (1, 1))
aff = (1.0 / 255.0, -0.5)
h1 = K.conv2d_fwd(x0, w1, g1, bias=b1, act="relu", in_affine=aff)
w2 = (torch.randn(64, 2, 2, 32, device=dev) * 0.1).to(bf)
b2 = torch.randn(64, device=dev) * 0.1
g2 = K.conv_geom(h1.shape, w2.shape, (1, 1), (0, 0), (1, 1))
rng = HF.rng_state(dev)
yp, am = K.conv2d_fwd_pool(h1, w2, g2, bias=b2, act="relu", drop_p=0.01, rng=rng, salt=3)
yc = K.conv2d_fwd(h1, w2, g2, bias=b2, act="relu")
yr, amr = K.maxpool2d_fwd(yc, (2, 2), (2, 2), (0, 0), drop_p=0.01, rng=rng, salt=3)
print("fwd_pool max|diff| vs unfused", (yp.float() - yr.float()).abs().max().item(), flush=True)
dy = (torch.randn(B, 26, 26, 64, device=dev) * 0.1).to(bf)
dw2 = torch.zeros(64, 128, device=dev)
db2 = torch.zeros(64, device=dev)
dw1 = torch.zeros(32, 4, device=dev)
db1 = torch.zeros(32, device=dev)
prev = (x0, g1, dw1, db1, h1, K.act_id("relu"), aff)
r = K.conv2d_bwd_pair(dy, w2, g2, h1, dw2, db2, prev=prev)
print("bwd_pair ->", "fused" if r is None else r, flush=True)
# numerics of the pair against torch fp32
torch.cuda.synchronize()
for t in (dw2, db2, dw1, db1):
    t.zero_()
K.conv2d_bwd_pair(dy, w2, g2, h1, dw2, db2, prev=prev)
hf = h1.float().permute(0, 3, 1, 2).requires_grad_(True)
w2f = w2.float().permute(0, 3, 1, 2).requires_grad_(True)
out = torch.nn.functional.conv2d(hf, w2f)
out.backward(dy.float().permute(0, 3, 1, 2))
ref_dw2 = w2f.grad.permute(0, 2, 3, 1).reshape(64, -1)
print("dw2 rel err", ((dw2 - ref_dw2).norm() / ref_dw2.norm()).item(), flush=True)
dh = hf.grad * (h1.float().permute(0, 3, 1, 2) > 0)
print("db1 rel err", ((db1 - dh.sum((0, 2, 3))).norm() / dh.sum((0, 2, 3)).norm()).item(), flush=True)

t_fwd1 = timeit(lambda: K.conv2d_fwd(x0, w1, g1, bias=b1, act="relu", in_affine=aff, out=h1))
t_fwd2 = timeit(lambda: K.conv2d_fwd_pool(h1, w2, g2, bias=b2, act="relu", drop_p=0.01, rng=rng, salt=3))
t_pair = timeit(lambda: K.conv2d_bwd_pair(dy, w2, g2, h1, dw2, db2, prev=prev))
t_dg = timeit(lambda: K.conv2d_dgrad_fused_wgrad(dy, w2, g2, h1, "relu", None, 0, x0, g1, dw1, db1, in_affine=aff))
t_wg = timeit(lambda: K.conv2d_wgrad(dy, h1, g2, dw2, dbias=db2))
print(f"dgrad+wgrad0 alone {t_dg:.2f} us  wgrad alone {t_wg:.2f} us", flush=True)
z = torch.zeros(1024, device=dev)
t_nop = timeit(lambda: z.zero_())
print(f"B={B} tiny-kernel {t_nop:.2f} us  conv1_direct_fwd {t_fwd1:.2f} us  conv2_fwd_pool {t_fwd2:.2f} us  conv2_bwd_pair {t_pair:.2f} us",
      flush=True)
