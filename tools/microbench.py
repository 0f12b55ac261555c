"""Per-op timing of the MNIST (E3) layer kernels at a given batch: mean us over N launches
(events around a loop, no host sync inside).  args: B [N]"""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hops_examples_amd.ops import kernels as K
B = int(sys.argv[1]); N = int(sys.argv[2]) if len(sys.argv) > 2 else 200
dev = torch.device("cuda", 0)
bf = torch.bfloat16
torch.manual_seed(0)
x0 = torch.randint(0, 256, (B, 28, 28, 1), dtype=torch.uint8, device=dev)
xn = K.u8_normalize(x0, 1 / 255, 0.0)
w1 = (torch.randn(32, 2, 2, 1, device=dev) * 0.3).to(bf)
w2 = (torch.randn(64, 2, 2, 32, device=dev) * 0.1).to(bf)
b1 = torch.zeros(32, device=dev); b2 = torch.zeros(64, device=dev)
g1 = K.conv_geom(xn.shape, w1.shape, (1, 1), (0, 0), (1, 1))
h1 = K.conv2d_fwd(xn, w1, g1, bias=b1, act=1)
g1u = K.conv_geom(x0.shape, w1.shape, (1, 1), (0, 0), (1, 1))
g2 = K.conv_geom(h1.shape, w2.shape, (1, 1), (0, 0), (1, 1))
h2 = K.conv2d_fwd(h1, w2, g2, bias=b2, act=1)
p, am = K.maxpool2d_fwd(h2, (2, 2), (2, 2), (0, 0))
flat = p.reshape(B, -1)
wf1 = (torch.randn(128, flat.shape[1], device=dev) * 0.01).to(bf); bf1 = torch.zeros(128, device=dev)
f1 = K.linear_fwd(flat, wf1, bf1, act=1)
wf2 = (torch.randn(10, 128, device=dev) * 0.1).to(bf); bf2 = torch.zeros(10, device=dev)
dy2 = torch.randn(B, 64 * 0 + h2.shape[1], h2.shape[2], 64, device=dev).to(bf)
dyp = torch.randn_like(p)
dw2 = torch.zeros(64, 2 * 2 * 32, device=dev); db2 = torch.zeros(64, device=dev)
dw1 = torch.zeros(32, 4, device=dev); db1 = torch.zeros(32, device=dev)
dh1 = torch.randn_like(h1)
dwf1 = torch.zeros(128, flat.shape[1], device=dev)
df1 = torch.randn(B, 128, device=dev).to(bf)
ops = {
    "u8_norm": lambda: K.u8_normalize(x0, 1 / 255, 0.0),
    "conv1_fwd": lambda: K.conv2d_fwd(xn, w1, g1, bias=b1, act=1),
    "conv2_fwd": lambda: K.conv2d_fwd(h1, w2, g2, bias=b2, act=1),
    "pool_fwd": lambda: K.maxpool2d_fwd(h2, (2, 2), (2, 2), (0, 0)),
    "fc1_fwd": lambda: K.linear_fwd(flat, wf1, bf1, act=1),
    "fc1_dgrad": lambda: K.linear_dgrad(df1, wf1, y=f1, act=1),
    "fc1_wgrad": lambda: K.linear_wgrad(df1, flat, dwf1, y=f1, act=1),
    "pool_bwd": lambda: K.maxpool2d_bwd(dyp, am, h2.shape, (2, 2), (2, 2), (0, 0)),
    "conv2_dgrad": lambda: K.conv2d_dgrad(dy2, w2, g2, yprev=h1, act_prev=1, y=h2, act=1),
    "conv2_dgrad_cs": lambda: K.conv2d_dgrad(dy2, w2, g2, yprev=h1, act_prev=1, y=h2, act=1, colsum=db1),
    "conv2_dgrad_fused": lambda: K.conv2d_dgrad_fused_wgrad(dy2, w2, g2, h1, 1, h2, 1, x0, g1u, dw1, db1,
                                                            in_affine=(1 / 255, -0.5)),
    "conv2_wgrad": lambda: K.conv2d_wgrad(dy2, h1, g2, dw2, dbias=db2, y=h2, act=1),
    "conv1_wgrad": lambda: K.conv2d_wgrad(dh1, xn, g1, dw1, dbias=db1, y=h1, act=1),
}
res = {}
only = os.environ.get("MB_ONLY")
for name, fn in ops.items():
    if only and name not in only.split(","):
        continue
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(N):
        fn()
    e.record()
    torch.cuda.synchronize()
    res[name] = round(s.elapsed_time(e) * 1000 / N, 2)
print(json.dumps({"B": B, "us": res}), flush=True)
