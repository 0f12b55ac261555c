"""Phase timing of the fused Dense->head kernel (loss.hip mlp_head_k) at the flagship shape:
stamps 0-2 from workgroup 0 (start, MFMA done, atomics done), 3-9 from the last workgroup."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hops_examples_amd.ops import _C, kernels as K
dev = torch.device("cuda", 0)
B, Kd, N1, C = 32, 10816, 128, 10
x = torch.randn(B, Kd, device=dev).to(torch.bfloat16)
w1 = (torch.randn(N1, Kd, device=dev) / Kd ** 0.5).to(torch.bfloat16)
b1 = torch.zeros(N1, device=dev)
w2 = (torch.randn(C, N1, device=dev) / N1 ** 0.5).to(torch.bfloat16)
b2 = torch.zeros(C, device=dev)
t = torch.randint(0, C, (B,), device=dev)
y = torch.empty(B, N1, device=dev, dtype=torch.bfloat16)
lg = torch.empty(B, C, device=dev, dtype=torch.bfloat16)
dw2 = torch.zeros(C, N1, device=dev); db2 = torch.zeros(C, device=dev)
loss = torch.empty(1, device=dev); corr = torch.empty(1, device=dev, dtype=torch.int32)
dbg = torch.zeros(16, device=dev, dtype=torch.int64)
f = lambda: K.mlp_head(x, w1, b1, "relu", y, 0, lg, t, w2, b2, dw2, db2, 1.0 / B, loss, corr)
for _ in range(20):
    f()
torch.cuda.synchronize()
_C.ext().mlp_head_debug(dbg.data_ptr())
res = []
for _ in range(20):
    dbg.zero_()
    f()
    torch.cuda.synchronize()
    d = dbg.cpu().tolist()
    res.append([(d[i] - d[0]) / 100.0 for i in range(10)])
_C.ext().mlp_head_debug(0)
med = [sorted(r[i] for r in res)[len(res) // 2] for i in range(10)]
names = ["start", "wg0_mfma_done", "wg0_atomics_done", "last_acquired", "ws_read_y_stored", "w2_staged",
         "logits_done", "loss_done", "dw2_done", "end"]
print(json.dumps({n: round(v, 2) for n, v in zip(names, med)}), flush=True)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(200):
    f()
b.record(); torch.cuda.synchronize()
print(json.dumps({"us_per_launch_back_to_back": round(a.elapsed_time(b) * 1000 / 200, 2)}))
