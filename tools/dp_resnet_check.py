"""Multi-rank check of a CIFAR ResNet-20 (8-channel padded image stem, BatchNorm, identity and
projection shortcuts) trained through DataParallel with the gradient exchange OVERLAPPED with the
backward: per-bucket all-reduces launched from hooks.grad_ready on the process-group path
(HOPSX_DPR_MODE=pg, p2p off) or per-bucket P2P reduce-scatters under the fused zero-copy step
(HOPSX_DPR_MODE=p2p).  Buckets are forced small so the model splits into several.

Run under torch.distributed.run with N ranks (ranks may share one GPU: gloo carries the process group).
Checks after a few eager + graph steps: the replicas' fp32 masters and bf16 compute weights are
bit-identical (DataParallel.verify_replicas) and the stem weight (the last gradient of the backward,
handed to the arena by _PadCinFn) moved identically on every rank.  Rank 0 prints one JSON line
prefixed DPRESNET.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

MODE = os.environ.get("HOPSX_DPR_MODE", "pg")
os.environ.setdefault("HOPSX_P2P", "0" if MODE == "pg" else "1")
os.environ.setdefault("HOPSX_DP_MIN_SPLIT_MB", "0")
os.environ.setdefault("HOPSX_DP_BUCKET_MB", "0.25")

import torch  # noqa: E402

from hops_examples_amd import optim  # noqa: E402
from hops_examples_amd.models.resnet import cifar_resnet  # noqa: E402
from hops_examples_amd.parallel import dist as hdist  # noqa: E402
from hops_examples_amd.parallel.dp import DataParallel  # noqa: E402
from hops_examples_amd.runtime.arena import ParamArena  # noqa: E402
from hops_examples_amd.runtime.step import TrainStep  # noqa: E402


def main():
    rank, _, world = hdist.init()
    dev = hdist.device()
    torch.manual_seed(5)
    m = cifar_resnet(20).to(dev)
    ParamArena.from_module(m, dev)
    opt = optim.SGD(m, lr=0.05, momentum=0.9)
    dp = DataParallel(m)
    st = TrainStep(m, opt, "sparse_ce", dp=dp, graph=dev.type == "cuda", warmup=2)
    res = {"world": world, "mode": MODE, "path": dp.path, "buckets": len(dp.buckets), "overlap": dp.overlap,
           "rs_mode": getattr(dp, "_rs_mode", False)}
    assert len(dp.buckets) > 1, dp.buckets
    if MODE == "pg":
        assert dp.overlap and dp._oneshot is None, (dp.overlap, dp.path)
    else:
        assert dp.path.endswith("-zerocopy-overlap"), dp.path
    rs_calls = []
    if MODE != "pg":
        # per-bucket ownership: every rank reduces its slice of EVERY bucket (the tail then updates pieces)
        orig_rs = dp._oneshot.dp_rs

        def logged(grad, lo, hi, blocks, stream):
            rs_calls.append((int(lo), int(hi)))
            return orig_rs(grad, lo, hi, blocks, stream)

        dp._oneshot.dp_rs = logged
    g = torch.Generator(device="cpu").manual_seed(200 + rank)  # every rank its own batch
    x = torch.randint(0, 256, (4, 16, 32, 32, 3), dtype=torch.uint8, generator=g).to(dev)
    y = torch.randint(0, 10, (4, 16), generator=g).to(dev)
    stem = m.stem.conv.weight
    w0 = stem.detach().clone()
    for i in range(6):  # 2 eager warm-up steps, the capture, then replays
        r = st(x[i % 4], y[i % 4])
    torch.cuda.synchronize() if dev.type == "cuda" else None
    res["loss"] = round(float(r["loss"].reshape(-1)[0]), 4)
    v = dp.verify_replicas()
    res["replicas_identical"] = v["identical"]
    assert v["identical"], v
    moved = float((stem.detach() - w0).abs().max())
    res["stem_moved"] = moved
    assert moved > 0.0  # the stem gradient reached the update
    if MODE != "pg":
        own = dp.owner_slices()[rank]
        per_bucket = []
        for lo, hi, _ in dp.buckets:
            mine = sum(max(0, min(hi, x.stop) - max(lo, x.start)) for x in own)
            per_bucket.append(mine)
        res[f"rank{rank}_owned_per_bucket"] = per_bucket
        res[f"rank{rank}_dp_rs_per_step"] = len(set(rs_calls))
        assert all(v > 0 for v in per_bucket), per_bucket  # a share of every bucket
        assert len(set(rs_calls)) == len(dp.buckets), (rs_calls, dp.buckets)
        objs = [None] * world
        torch.distributed.all_gather_object(objs, res)
        for o in objs:
            res.update(o)
    dp.close()
    if rank == 0:
        print("DPRESNET " + json.dumps(res), flush=True)
    hdist.shutdown()


if __name__ == "__main__":
    main()
