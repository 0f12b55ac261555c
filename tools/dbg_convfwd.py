"""Phase stamps (100 MHz wall clock, wave 0 of each workgroup) of the flagship's conv2 forward
(conv_fwd_mfma_k POOL) and backward pair (conv_bwd_pair_k) at batch 32.  Prints, per launch, the
spread of workgroup start times and the mean / max of each phase."""
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


def stamps(fn, names):
    ext = _C.ext()
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t = np.array(ext.wgrad_debug_times(2048 * 4), dtype=np.int64).reshape(-1, 4)
    return t


def report(title, t, rows, names):
    t = t[rows]
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    ph = (t - t0) / 100.0
    print(f"== {title}: {len(t)} WGs, start spread {ph[:, 0].max():.2f} us, last end {ph[:, 3].max():.2f} us")
    for i, n in enumerate(names):
        d = ph[:, i + 1] - ph[:, i]
        print(f"   {n:24s} mean {d.mean():6.2f}  max {d.max():6.2f} us")


t = stamps(lambda: K.conv2d_fwd_pool(h1, w2, g2, bias=b2, act="relu", drop_p=0.01, rng=rng, salt=3), None)
n = (B * 13 * 13 * 4 + 15) // 16
nwg = (n + 7) // 8
report("conv2 fwd+pool", t, slice(0, nwg), ["stage weights", "A loads + MFMA (u0)", "epilogue + stores"])
t = stamps(lambda: K.conv2d_bwd_pair(dy, w2, g2, h1, dw2, db2, prev=prev), None)
Md = B * 27 * 27
nA = min(512, ((Md + 15) // 16 + 7) // 8)
report("bwd pair: dgrad part", t, slice(0, nA), ["stage weights", "loop", "reduce + atomics"])
report("bwd pair: wgrad part", t, slice(nA, 2048), ["loop", "lds reduce", "atomics"])
# the two halves of the pair as separate launches (interference check)
t = stamps(lambda: K.conv2d_dgrad_fused_wgrad(dy, w2, g2, h1, "relu", None, 0, x0, g1, dw1, db1, in_affine=aff), None)
report("dgrad alone (fused wgrad0)", t, slice(0, nA), ["stage weights", "loop", "reduce + atomics"])
t = stamps(lambda: K.conv2d_wgrad(dy, h1, g2, dw2, dbias=db2), None)
report("wgrad alone", t, slice(0, 2048), ["loop", "lds reduce", "atomics"])
