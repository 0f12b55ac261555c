"""Debug: A (fused P2P step) vs C (P2P all-reduce + optimizer) vs B (process-group all-reduce),
compared after every step from the same RNG state.  torchrun, ranks sharing one GPU, gloo."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("HOPSX_P2P", "1")
import torch  # noqa: E402

from hops_examples_amd import optim  # noqa: E402
from hops_examples_amd.models.mnist import MirroredMnistCNN  # noqa: E402
from hops_examples_amd.ops.functional import rng_state  # noqa: E402
from hops_examples_amd.parallel import dist as hdist  # noqa: E402
from hops_examples_amd.parallel.dp import DataParallel  # noqa: E402
from hops_examples_amd.runtime.arena import ParamArena  # noqa: E402
from hops_examples_amd.runtime.step import TrainStep  # noqa: E402


def build(dev, p2p, fused):
    os.environ["HOPSX_P2P_FUSED"] = "1" if fused else "0"
    torch.manual_seed(7)
    m = MirroredMnistCNN().to(dev)
    ParamArena.from_module(m, dev)
    opt = optim.SGD(m, lr=0.05, momentum=0.5)
    dp = DataParallel(m, p2p=p2p)
    st = TrainStep(m, opt, "sparse_ce", dp=dp, warmup=2, steps_per_execution=4, graph=os.environ.get("G", "1") == "1")
    m.salt_src = m
    return opt, dp, st


def main():
    rank, _, world = hdist.init()
    dev = hdist.device()
    B, nb = 32, 16
    g = torch.Generator(device="cpu").manual_seed(100 + rank)
    xs = torch.randint(0, 256, (nb, B, 28, 28, 1), dtype=torch.uint8, generator=g).to(dev)
    ys = torch.randint(0, 10, (nb, B), dtype=torch.int64, generator=g).to(dev)
    os.environ["HOPSX_OPT_KIND"] = "sgd"
    runs = {"A": build(dev, None, True), "C": build(dev, None, False), "B": build(dev, False, False),
            "B2": build(dev, False, False)}
    mods = [list(r[0].arena.params[0]._hx_arena.params) for r in runs.values()]
    ms = [r[2].model for r in runs.values()]
    for other in ms[1:]:  # dropout salts come from a per-instance counter: share A's
        for ma, mo in zip(ms[0].modules(), other.modules()):
            if hasattr(ma, "salt"):
                mo.salt = ma.salt
    if rank == 0:
        print({k: v[1].path for k, v in runs.items()}, flush=True)
    rng0 = rng_state(dev).clone()
    hist = {k: [] for k in runs}
    init = runs["A"][0].arena.master.clone()
    for k, (opt, dp, st) in runs.items():
        rng_state(dev).copy_(rng0)
        for i in range(10):
            st.step_resident(xs, ys)
            torch.cuda.synchronize()
            hist[k].append(opt.arena.master.clone())

    def rel(x, y):
        return float((x - y).norm() / (y - init).norm())

    for i in range(10):
        a, c, b, b2 = hist["A"][i], hist["C"][i], hist["B"][i], hist["B2"][i]
        if rank == 0:
            print(f"step {i}: rel A-C {rel(a, c):.3e} C-B {rel(c, b):.3e} A-B {rel(a, b):.3e} B2-B {rel(b2, b):.3e}",
                  flush=True)
    for k, (opt, dp, st) in runs.items():
        dp.close()
    hdist.shutdown()


if __name__ == "__main__":
    main()
