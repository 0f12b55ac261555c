"""Phase timestamps (100 MHz wall clock) of conv_wgrad_mfma_k workgroups at the MNIST conv2 shape."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["HOPSX_PHASE_DBG"] = "1"
import numpy as np
import torch
from hops_examples_amd.ops import kernels as K
from hops_examples_amd.ops import _C
dev = torch.device("cuda", 0); bf = torch.bfloat16
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
h1 = torch.randn(B, 27, 27, 32, device=dev).to(bf)
dy = torch.randn(B, 26, 26, 64, device=dev).to(bf)
y = torch.relu(torch.randn(B, 26, 26, 64, device=dev)).to(bf)
g = K.conv_geom(h1.shape, (64, 2, 2, 32), (1, 1), (0, 0), (1, 1))
dw = torch.zeros(64, 128, device=dev); db = torch.zeros(64, device=dev)
for _ in range(20):
    K.conv2d_wgrad(dy, h1, g, dw, dbias=db, y=y, act=1)
torch.cuda.synchronize()
t = np.array(_C.ext().wgrad_debug_times(2048 * 4), dtype=np.int64).reshape(-1, 4)
t = t[t[:, 0] > 0]
t0 = t[:, 0].min()
ph = (t - t0) / 100.0  # us
print("WGs", len(t))
print("start  spread us: %.2f" % (ph[:, 0].max()))
print("loop   mean/max us: %.2f / %.2f" % ((ph[:, 1] - ph[:, 0]).mean(), (ph[:, 1] - ph[:, 0]).max()))
print("lds    mean/max us: %.2f / %.2f" % ((ph[:, 2] - ph[:, 1]).mean(), (ph[:, 2] - ph[:, 1]).max()))
print("atomic mean/max us: %.2f / %.2f" % ((ph[:, 3] - ph[:, 2]).mean(), (ph[:, 3] - ph[:, 2]).max()))
print("end max us: %.2f" % ph[:, 3].max())
