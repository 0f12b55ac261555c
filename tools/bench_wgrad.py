"""Per-layer timing of the ResNet-50 conv weight gradients: the glds kernel (direct binding), the
``conv2d_wgrad`` dispatch, and PyTorch's own bf16 channels-last weight gradient for scale.

usage (GPU): python tools/bench_wgrad.py [--batch 64] [--iters 20]
Prints one line per geometry with us / TFLOP/s and the step total (x the layer's count in the net).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hops_examples_amd.ops import _C  # noqa: E402
from hops_examples_amd.ops import kernels as K  # noqa: E402

# (H_in, C, CO, k, stride, count in ResNet-50 v1.5)
LAYERS = [
    (56, 64, 64, 1, 1, 1), (56, 64, 64, 3, 1, 3), (56, 64, 256, 1, 1, 4), (56, 256, 64, 1, 1, 2),
    (56, 256, 128, 1, 1, 1), (56, 128, 128, 3, 2, 1), (28, 128, 512, 1, 1, 4), (56, 256, 512, 1, 2, 1),
    (28, 512, 128, 1, 1, 3), (28, 128, 128, 3, 1, 3),
    (28, 512, 256, 1, 1, 1), (28, 256, 256, 3, 2, 1), (14, 256, 1024, 1, 1, 6), (28, 512, 1024, 1, 2, 1),
    (14, 1024, 256, 1, 1, 5), (14, 256, 256, 3, 1, 5),
    (14, 1024, 512, 1, 1, 1), (14, 512, 512, 3, 2, 1), (7, 512, 2048, 1, 1, 3), (14, 1024, 2048, 1, 2, 1),
    (7, 2048, 512, 1, 1, 2), (7, 512, 512, 3, 1, 2),
]


def timeit(fn, iters):
    """GPU time per call: `iters` calls captured into one hipGraph (eager launches would time the
    Python launch overhead, ~20-30 us a call, not the kernel)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(iters):
            fn()
    graph.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    graph.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--torch", action="store_true", help="also time PyTorch's weight gradient")
    ap.add_argument("--glds-only", action="store_true", help="skip the conv2d_wgrad dispatch timing")
    ap.add_argument("--only", default="", help="H,C,CO,k,s of the one layer to run (profiling)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    tot = {"glds": 0.0, "dispatch": 0.0, "torch": 0.0}
    only = tuple(int(v) for v in a.only.split(",")) if a.only else None
    for (H, C, CO, k, s, n) in LAYERS:
        if only and (H, C, CO, k, s) != only:
            continue
        B = a.batch
        x = torch.randn(B, H, H, C, device=dev).to(bf)
        g = K.conv_geom(x.shape, (CO, k, k, C), (s, s), (k // 2, k // 2), (1, 1))
        dy = torch.randn(B, g[4], g[5], CO, device=dev).to(bf)
        dw = torch.zeros(CO, k * k * C, device=dev)
        flop = 2.0 * B * g[4] * g[5] * CO * k * k * C
        row = {"H": H, "C": C, "CO": CO, "k": k, "s": s, "n": n}
        if _C.ext().conv_wgrad_glds_ok(g):
            us = timeit(lambda: _C.ext().conv2d_wgrad_glds(K.ptr(dy), K.ptr(x), g, K.ptr(dw), 1, K.stream()), a.iters)
            row["glds_us"] = round(us, 1)
            row["glds_tf"] = round(flop / us / 1e6, 1)
            tot["glds"] += us * n
        us = timeit(lambda: K.conv2d_wgrad(dy, x, g, dw), a.iters) if not a.glds_only else 0.0
        row["disp_us"] = round(us, 1)
        row["disp_tf"] = round(flop / us / 1e6, 1) if us else 0.0
        tot["dispatch"] += us * n
        if a.torch:
            xt = x.permute(0, 3, 1, 2)
            dyt = dy.permute(0, 3, 1, 2)
            us = timeit(lambda: torch.ops.aten.convolution_backward(
                dyt, xt, torch.empty(CO, C, k, k, device=dev, dtype=bf).to(memory_format=torch.channels_last),
                None, [s, s], [k // 2, k // 2], [1, 1], False, [0, 0], 1, [False, False, True]), a.iters)
            row["torch_us"] = round(us, 1)
            row["torch_tf"] = round(flop / us / 1e6, 1)
            tot["torch"] += us * n
        print(json.dumps(row), flush=True)
    print(json.dumps({"batch": a.batch, "step_total_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
