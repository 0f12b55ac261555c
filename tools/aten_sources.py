"""Which Python lines launch PyTorch's own kernels (aten fill / copy / cast / elementwise) inside a
training step: torch.profiler with stacks over a few eager TrainStep steps of a model, grouped by op
and the innermost hops_examples_amd frame.
usage (GPU): python tools/aten_sources.py [resnet20|resnet50] [batch]"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hops_examples_amd import optim  # noqa: E402
from hops_examples_amd.models.resnet import cifar_resnet, resnet50  # noqa: E402
from hops_examples_amd.runtime.arena import ParamArena  # noqa: E402
from hops_examples_amd.runtime.step import TrainStep  # noqa: E402

WATCH = ("aten::fill_", "aten::zero_", "aten::copy_", "aten::to", "aten::_to_copy", "aten::add_", "aten::add",
         "aten::mul", "aten::mul_", "aten::zeros", "aten::zeros_like", "aten::contiguous", "aten::clone", "aten::cat",
         "aten::sub", "aten::div", "aten::sum", "aten::index_put_", "aten::masked_fill_", "aten::where")


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "resnet20"
    dev = torch.device("cuda", 0)
    if which == "resnet50":
        B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
        m, H, ncls = resnet50().to(dev), 224, 1000
        opt_fn = lambda m: optim.RMSprop(m, lr=0.2)  # noqa: E731
    else:
        B = int(sys.argv[2]) if len(sys.argv) > 2 else 128
        m, H, ncls = cifar_resnet(20).to(dev), 32, 10
        opt_fn = lambda m: optim.SGD(m, lr=0.1, momentum=0.9)  # noqa: E731
    ParamArena.from_module(m, dev)
    opt = opt_fn(m)
    st = TrainStep(m, opt, "sparse_ce", graph=False)
    x = torch.randint(0, 256, (B, H, H, 3), dtype=torch.uint8, device=dev)
    y = torch.randint(0, ncls, (B,), device=dev)
    for _ in range(3):
        st(x, y)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
        for _ in range(2):
            st(x, y)
        torch.cuda.synchronize()
    hits = collections.Counter()
    for ev in prof.events():
        if ev.name not in WATCH:
            continue
        frames = [f for f in (ev.stack or []) if "hops_examples_amd" in f or "tools/" in f]
        where = frames[0] if frames else "(no hopsx frame)"
        hits[(ev.name, where, str(ev.input_shapes)[:80])] += 1
    print(f"# {which} B={B}: aten ops per 2 eager steps, by innermost hopsx frame")
    for (name, where, shp), n in sorted(hits.items(), key=lambda kv: -kv[1]):
        print(f"{n:4d}  {name:18s} {where[-90:]:90s} {shp}")


if __name__ == "__main__":
    main()
