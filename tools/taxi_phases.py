"""Phase timestamps of the fused taxi step kernel (HOPSX_PHASE_DBG=1; wall clock, 100 MHz).

v2 (taxi_step.hip, default): one launch of N steps; prints the launch prologue, the mean step time
((end - staged) / N, write-back included) and the phase boundaries of the launch's LAST step.
v1 (widedeep_step.hip, HOPSX_TAXI_KERNEL=v1): one-step launches, the mean of each boundary.
usage: python tools/taxi_phases.py [N]"""
import os
import sys

os.environ["HOPSX_PHASE_DBG"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hops_examples_amd.models import widedeep as WD  # noqa: E402
from hops_examples_amd.runtime.arena import ParamArena  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 32
dev = torch.device("cuda", 0)
B, nb = 40, 64
dense, cat, label = WD.synth_taxi(nb * B, seed=3, device=dev)
m = WD.TaxiWideDeep().to(dev)
ParamArena.from_module(m, dev)
fs = WD.FusedWideDeepStep(m, WD.make_optimizer(m))
xs, ys = (dense.view(nb, B, -1), cat.view(nb, B, -1)), label.view(nb, B, 1)
print(f"kernel {fs.kernel}")
if fs.kernel == "v2":
    # stamps: 0 launch, 1 prologue done, 7 last step start, 2 FWD, 3 B3, 4 B2, 5 B1, 6 B0 (ends), 19 end
    rows = [("prologue", 0, 1), ("per step (mean)", None, None), ("FWD  fwd+loss", 7, 2), ("B3   dX3 dW3 dW4", 2, 3),
            ("B2   dX2 dW2", 3, 4), ("B1   dX1 dW1", 4, 5), ("B0   dW0 FTRL", 5, 6), ("write-back", 6, 19),
            ("  fwd: gather+L0", 7, 8), ("  fwd: L1", 8, 9), ("  fwd: L2", 9, 10), ("  fwd: L3", 10, 11),
            ("  fwd: loss+G4+dW4", 11, 12), ("  fwd: bar wait", 12, 2), ("  B3 w0: dX3", 2, 13),
            ("  B3 w0: marks", 13, 14), ("  B3 w3: dW3 x2", 2, 15), ("  B1 w0: dX1", 4, 16),
            ("  B1 w3: put+dW1 x5", 4, 17), ("  B0 w0: dW0+FTRL", 5, 18),
            ("  wb: loss reduce", 6, 22), ("  wb: w fill", 22, 23), ("  wb: w put", 23, 24), ("  wb: w copy", 24, 26),
            ("  wb: s put", 26, 27), ("  wb: s copy", 27, 29), ("  wb: wide", 29, 19)]
    fs.steps_per_execution = N
    acc = {}
    for it in range(12):
        fs.run_resident(xs, ys, N)
        torch.cuda.synchronize()
        t = fs.dbg.cpu().tolist()
        if it >= 2:
            for name, a0, a1 in rows:
                v = (t[19] - t[1]) / N if a0 is None else t[a1] - t[a0]
                acc.setdefault(name, []).append(v / 100.0)
            acc.setdefault("shader clock GHz", []).append(100.0 * (t[21] - t[20]) / max(1, t[6] - t[1]) / 1000.0)
    for k, v in acc.items():
        print(f"{k:20s} {sum(v) / len(v):8.3f} " + ("" if "GHz" in k else "us"))
    print(f"(phase rows: the last of the launch's {N} steps; clock = memtime ticks per wall tick x 100 MHz)")
else:
    names = {0: "start", 1: "staged", 10: "loss"}
    names.update({2 + l: f"fwd{l}" for l in range(8)})
    names.update({11 + l: f"bwd{l}" for l in range(8)})
    names[19] = "end"
    acc = {}
    for it in range(30):
        fs.step_resident(xs, ys, graph=False)
        torch.cuda.synchronize()
        t = fs.dbg.cpu().tolist()
        if it >= 10:
            for k in range(1, 20):
                if t[k] and t[0]:
                    acc.setdefault(k, []).append((t[k] - t[0]) / 100.0)
    for k in sorted(acc):
        v = acc[k]
        print(f"{names[k]:8s} t+{sum(v) / len(v):7.2f} us")
