"""Per-layer timing of the ResNet-50 convolution GEMMs through the hopsx dispatch (forward, dgrad,
weight gradient), next to PyTorch's own bf16 channels-last convolution (MIOpen / hipBLASLt) for scale
(``--torch``: t_fwd / t_dgrad / t_wgrad and the hopsx / PyTorch ratios *_x).
Run it twice — default and HOPSX_DISABLE=gg — to compare the gg engine with gemm_core.h's.

usage (GPU): python tools/bench_conv_gemm.py [--batch 64] [--iters 20] [--torch]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hops_examples_amd.ops import kernels as K  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_wgrad import LAYERS, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--torch", action="store_true")
    ap.add_argument("--only", default="", help="H,C,CO,k,s of the one layer to run (profiling)")
    a = ap.parse_args()
    only = tuple(int(v) for v in a.only.split(",")) if a.only else None
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    tot = {}
    for (H, C, CO, k, s, n) in LAYERS:
        if only and (H, C, CO, k, s) != only:
            continue
        B = a.batch
        x = torch.randn(B, H, H, C, device=dev).to(bf)
        w = (torch.randn(CO, k, k, C, device=dev) * 0.05).to(bf)
        g = K.conv_geom(x.shape, w.shape, (s, s), (k // 2, k // 2), (1, 1))
        dy = torch.randn(B, g[4], g[5], CO, device=dev).to(bf)
        dw = torch.zeros(CO, k * k * C, device=dev)
        flop = 2.0 * B * g[4] * g[5] * CO * k * k * C
        row = {"H": H, "C": C, "CO": CO, "k": k, "s": s, "n": n}
        for name, fn in (("fwd", lambda: K.conv2d_fwd(x, w, g)), ("dgrad", lambda: K.conv2d_dgrad(dy, w, g)),
                         ("wgrad", lambda: K.conv2d_wgrad(dy, x, g, dw))):
            us = timeit(fn, a.iters)
            row[name] = round(us, 1)
            row[name + "_tf"] = round(flop / us / 1e6, 1)
            tot[name] = tot.get(name, 0.0) + us * n
        if a.torch:
            xt = x.permute(0, 3, 1, 2)
            wt = w.permute(0, 3, 1, 2)
            dyt = dy.permute(0, 3, 1, 2)
            us = timeit(lambda: F.conv2d(xt, wt, stride=s, padding=k // 2), a.iters)
            row["t_fwd"] = round(us, 1)
            tot["t_fwd"] = tot.get("t_fwd", 0.0) + us * n
            us = timeit(lambda: torch.ops.aten.convolution_backward(
                dyt, xt, wt, None, [s, s], [k // 2, k // 2], [1, 1], False, [0, 0], 1, [True, False, False]), a.iters)
            row["t_dgrad"] = round(us, 1)
            tot["t_dgrad"] = tot.get("t_dgrad", 0.0) + us * n
            us = timeit(lambda: torch.ops.aten.convolution_backward(
                dyt, xt, wt, None, [s, s], [k // 2, k // 2], [1, 1], False, [0, 0], 1, [False, True, False]), a.iters)
            row["t_wgrad"] = round(us, 1)
            tot["t_wgrad"] = tot.get("t_wgrad", 0.0) + us * n
            for name in ("fwd", "dgrad", "wgrad"):
                row[name + "_x"] = round(row[name] / row["t_" + name], 2)
        print(json.dumps(row), flush=True)
    print(json.dumps({"batch": a.batch, "step_total_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
