"""GEMM / conv kernel efficiency: TFLOP/s of the MFMA kernels on square GEMMs and ResNet-50 conv
shapes (batch 64), measured with events around N back-to-back launches."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hops_examples_amd.ops import kernels as K
dev = torch.device("cuda", 0)
bf = torch.bfloat16
res = {}


def tm(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e-3


for M, N, Kd in [(4096, 4096, 4096), (8192, 8192, 8192), (16384, 4096, 4096)]:
    a = torch.randn(M, Kd, device=dev).to(bf); w = torch.randn(N, Kd, device=dev).to(bf)
    t = tm(lambda: K.linear_fwd(a, w))
    tt = tm(lambda: torch.matmul(a, w.t()))
    res[f"gemm_{M}x{N}x{Kd}"] = {"hopsx_tflops": round(2 * M * N * Kd / t / 1e12, 1),
                                 "torch_tflops": round(2 * M * N * Kd / tt / 1e12, 1)}
B = 64
for (H, C, CO, k, s) in [(56, 64, 64, 3, 1), (56, 64, 256, 1, 1), (28, 128, 128, 3, 1), (14, 256, 256, 3, 1),
                         (7, 512, 512, 3, 1), (56, 256, 128, 1, 1), (224, 3, 64, 7, 2)]:
    x = torch.randn(B, H, H, C, device=dev).to(bf)
    w = (torch.randn(CO, k, k, C, device=dev) * 0.05).to(bf)
    g = K.conv_geom(x.shape, w.shape, (s, s), (k // 2, k // 2), (1, 1))
    OH = g[4]
    fl = 2 * B * OH * OH * CO * k * k * C
    y = K.conv2d_fwd(x, w, g)
    dy = torch.randn_like(y)
    dw = torch.zeros(CO, k * k * C, device=dev)
    tf = tm(lambda: K.conv2d_fwd(x, w, g))
    td = tm(lambda: K.conv2d_dgrad(dy, w, g)) if C >= 8 else float("nan")
    tw = tm(lambda: K.conv2d_wgrad(dy, x, g, dw))
    xn = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
    wn = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
    tr = tm(lambda: torch.nn.functional.conv2d(xn, wn, stride=s, padding=k // 2))
    res[f"conv_{H}x{C}->{CO}_k{k}s{s}"] = {"fwd_tflops": round(fl / tf / 1e12, 1), "dgrad_tflops": round(fl / td / 1e12, 1),
                                           "wgrad_tflops": round(fl / tw / 1e12, 1),
                                           "miopen_fwd_tflops": round(fl / tr / 1e12, 1), "fwd_us": round(tf * 1e6, 1)}
print(json.dumps(res, indent=1), flush=True)
