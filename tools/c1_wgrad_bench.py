"""Time the one-channel input-layer weight gradient (conv.hip conv_wgrad_c1_k vs the channel-group
smallk kernel, HOPSX_DISABLE=c1_wgrad) at the E1 shape: batch 32, 28x28x1, 4x4, 32 channels."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hops_examples_amd.ops import kernels as K  # noqa: E402

dev = torch.device("cuda", 0)
STOP = os.environ.get("HOPSX_C1_STOP", "0")
for B, k, CO in ((32, 4, 32), (32, 2, 32), (32, 5, 16)):
    xu = torch.randint(0, 256, (B, 28, 28, 1), dtype=torch.uint8, device=dev)
    g = K.conv_geom(xu.shape, (CO, k, k, 1), (1, 1), (0, 0), (1, 1))
    dy = torch.randn(B, g[4], g[5], CO, device=dev).to(torch.bfloat16)
    y = torch.relu(torch.randn_like(dy.float())).to(torch.bfloat16)
    dw = torch.zeros(CO, k * k, device=dev)
    db = torch.zeros(CO, device=dev)
    res = {}
    for flag in ("", "c1_wgrad"):
        os.environ["HOPSX_DISABLE"] = flag
        for _ in range(5):
            K.conv2d_wgrad(dy, xu, g, dw, dbias=db, y=y, act="relu", in_affine=(1 / 255.0, -0.5))
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            K.conv2d_wgrad(dy, xu, g, dw, dbias=db, y=y, act="relu", in_affine=(1 / 255.0, -0.5))
        e1.record()
        torch.cuda.synchronize()
        res[flag or "c1"] = round(e0.elapsed_time(e1) / 200 * 1000, 2)
    print(f"B={B} k={k} CO={CO} stop={STOP}: us per call {res}")
