"""Phase timestamps (100 MHz wall clock) of the fused conv dgrad at the MNIST conv2 shape."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["HOPSX_PHASE_DBG"] = "1"
import numpy as np
import torch
from hops_examples_amd.ops import kernels as K
from hops_examples_amd.ops import _C
dev = torch.device("cuda", 0); bf = torch.bfloat16
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
x0 = torch.randint(0, 256, (B, 28, 28, 1), dtype=torch.uint8, device=dev)
h1 = torch.relu(torch.randn(B, 27, 27, 32, device=dev)).to(bf)
dy = torch.randn(B, 26, 26, 64, device=dev).to(bf)
w2 = (torch.randn(64, 2, 2, 32, device=dev) * 0.1).to(bf)
g1 = K.conv_geom(x0.shape, (32, 2, 2, 1), (1, 1), (0, 0), (1, 1))
g2 = K.conv_geom(h1.shape, (64, 2, 2, 32), (1, 1), (0, 0), (1, 1))
dw1 = torch.zeros(32, 4, device=dev); db1 = torch.zeros(32, device=dev)
for _ in range(20):
    K.conv2d_dgrad_fused_wgrad(dy, w2, g2, h1, 1, None, 0, x0, g1, dw1, db1, in_affine=(1 / 255, -0.5))
torch.cuda.synchronize()
t = np.array(_C.ext().wgrad_debug_times(2048 * 4), dtype=np.int64).reshape(-1, 4)
t = t[t[:, 0] > 0]
ph = (t - t[:, 0].min()) / 100.0
print("WGs", len(t), "start spread us %.2f" % ph[:, 0].max())
for i, n in enumerate(["stage", "loop", "reduce+atomics"]):
    d = ph[:, i + 1] - ph[:, i]
    print("%-15s mean %.2f max %.2f" % (n, d.mean(), d.max()))
print("end max us %.2f" % ph[:, 3].max())
