"""Flagship conv chain at batch 32: per-launch time (200 back-to-back launches, events) and
per-workgroup phase stamps (HOPSX_PHASE_DBG, wave 0 of each workgroup, 100 MHz) of
(a) input layer + conv2 + pool as two launches, (b) the fused launch (conv_mfma.hip IN0),
(c) the conv backward pair (conv2 dgrad + wgrad + input-layer wgrad)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["HOPSX_PHASE_DBG"] = "1"
import numpy as np
import torch

from hops_examples_amd.ops import _C
from hops_examples_amd.ops import functional as HF
from hops_examples_amd.ops import kernels as K

dev = torch.device("cuda", 0)
bf = torch.bfloat16
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
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
dy = (torch.randn(B, 26, 26, 64, device=dev) * 0.1).to(bf)
dw2 = torch.zeros(64, 128, device=dev)
db2 = torch.zeros(64, device=dev)
dw1 = torch.zeros(32, 4, device=dev)
db1 = torch.zeros(32, device=dev)
prev = (x0, g1, dw1, db1, h1, K.act_id("relu"), aff)


def timed(fn, n=200):
    for _ in range(10):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / n


def stamps(fn):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    return np.array(_C.ext().wgrad_debug_times(2048 * 4), dtype=np.int64).reshape(-1, 4)


def report(title, t, rows, names):
    t = t[rows]
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    ph = (t - t0) / 100.0
    print(f"== {title}: {len(t)} WGs, start spread {ph[:, 0].max():.2f} us, last end {ph[:, 3].max():.2f} us")
    for i, n in enumerate(names):
        d = ph[:, i + 1] - ph[:, i]
        print(f"   {n:24s} mean {d.mean():6.2f}  max {d.max():6.2f} us")


unf1 = lambda: K.conv2d_fwd(x0, w1, g1, bias=b1, act="relu", in_affine=aff)  # noqa: E731
unf2 = lambda: K.conv2d_fwd_pool(h1, w2, g2, bias=b2, act="relu", drop_p=0.01, rng=rng, salt=3)  # noqa: E731
fused = lambda: K.conv2d_fwd_pool_in(x0, w1, b1, "relu", g1, w2, g2, bias=b2, act="relu", drop_p=0.01,  # noqa: E731
                                     rng=rng, salt=3, in_affine=aff)
fused_nokeep = lambda: K.conv2d_fwd_pool_in(x0, w1, b1, "relu", g1, w2, g2, bias=b2, act="relu",  # noqa: E731
                                            drop_p=0.01, rng=rng, salt=3, in_affine=aff, keep_y1=False)
print(f"input layer alone {timed(unf1):.2f} us, conv2+pool alone {timed(unf2):.2f} us, "
      f"both {timed(lambda: (unf1(), unf2())):.2f} us, fused {timed(fused):.2f} us, "
      f"fused w/o y1 store {timed(fused_nokeep):.2f} us")
n = (B * 13 * 13 * 4 + 15) // 16
nwg = (n + 3) // 4
names = ["stage weights", "A loads + MFMA (u0)", "epilogue + stores"]
report("conv2 fwd+pool (unfused)", stamps(unf2), slice(0, nwg), names)
report("input layer + conv2 fwd+pool (fused)", stamps(fused), slice(0, nwg), names)
pair = lambda: K.conv2d_bwd_pair(dy, w2, g2, h1, dw2, db2, prev=prev)  # noqa: E731
print(f"bwd pair {timed(pair):.2f} us")
t = stamps(pair)
Md = B * 27 * 27
nA = min(512, ((Md + 15) // 16 + 7) // 8)
report("bwd pair: dgrad part", t, slice(0, nA), ["stage weights", "loop", "reduce + atomics"])
report("bwd pair: wgrad part", t, slice(nA, 2048), ["loop", "lds reduce", "atomics"])
