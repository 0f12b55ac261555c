"""1x1-conv weight gradient (dW[CO][C] += dY^T X, K = B*H*W) at ResNet-50 B=64 shapes: the hopsx
split-K MFMA kernel vs hipBLASLt (torch.mm) fp32-out and bf16-out."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hops_examples_amd.ops import kernels as K
dev = torch.device("cuda", 0)
bf = torch.bfloat16


def tm(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


res = {}
for (H, C, CO) in [(56, 64, 256), (56, 256, 64), (28, 512, 128), (28, 128, 512), (14, 1024, 256), (14, 256, 1024),
                   (7, 2048, 512), (7, 512, 2048)]:
    B = 64
    x = torch.randn(B, H, H, C, device=dev).to(bf)
    dy = torch.randn(B, H, H, CO, device=dev).to(bf)
    g = K.conv_geom(x.shape, (CO, 1, 1, C), (1, 1), (0, 0), (1, 1))
    dw = torch.zeros(CO, C, device=dev)
    Kd = B * H * H
    fl = 2.0 * Kd * C * CO
    t0 = tm(lambda: K.conv2d_wgrad(dy, x, g, dw))
    d2, x2 = dy.view(-1, CO), x.view(-1, C)
    t1 = tm(lambda: dw.add_(torch.mm(d2.t(), x2, out_dtype=torch.float32)))
    t2 = tm(lambda: dw.add_(torch.mm(d2.t(), x2)))
    res[f"{H}x{C}->{CO}"] = {"hopsx_us": round(t0, 1), "blaslt_f32out_us": round(t1, 1), "blaslt_bf16out_us": round(t2, 1),
                             "hopsx_tflops": round(fl / t0 / 1e6, 1), "best_lib_tflops": round(fl / min(t1, t2) / 1e6, 1)}
print(json.dumps(res, indent=1), flush=True)
