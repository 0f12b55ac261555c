"""Multi-rank check of the one-shot all-reduce (parallel/oneshot.py, csrc/comm/oneshot.hip).

Run under torch.distributed.run with N ranks; on a one-GPU box the ranks share the device
(HOPSX_DIST_BACKEND=gloo carries only the IPC-handle exchange and barriers).  Checks bitwise
equality with the rank-ordered fp32 sum for ragged sizes, repeated calls (epoch parity reuse),
hipGraph capture + replay, then times the kernel.  Rank 0 prints one JSON line.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hops_examples_amd.parallel import dist as hdist  # noqa: E402
from hops_examples_amd.parallel.oneshot import OneShotAllReduce  # noqa: E402


def inputs(n, world, it, dev):
    xs = []
    for r in range(world):
        g = torch.Generator(device="cpu").manual_seed(1000 * it + r)
        xs.append(torch.randn(n, generator=g).to(dev))
    ref = xs[0].clone()
    for r in range(1, world):
        ref += xs[r]
    return xs, ref


def main():
    rank, _, world = hdist.init()
    dev = hdist.device()
    ar = OneShotAllReduce(cap_bytes=8 << 20, device=dev)
    res = {"world": world, "checks": 0}
    modes = ("one_shot", "two_shot")
    for it, n in enumerate([1, 3, 4, 5, 257, 1000, 18866, 65536 + 7, 1394282, ar.cap]):
        for mode in modes:  # interleaved modes share the epoch/parity staging layout
            xs, ref = inputs(n, world, it, dev)
            x = xs[rank].clone()
            ar(x, mode=mode)
            torch.cuda.synchronize()
            ar.check()
            assert torch.equal(x, ref), (rank, n, mode, (x - ref).abs().max().item())
            res["checks"] += 1
    # out-of-place + repeated calls of the same size (double-buffer reuse)
    for it in range(20):
        xs, ref = inputs(4099, world, 100 + it, dev)
        out = torch.empty_like(ref)
        ar(xs[rank], out, mode=modes[it % 2])
        torch.cuda.synchronize()
        assert torch.equal(out, ref), (rank, it)
        res["checks"] += 1
    # hipGraph capture: the epoch lives on the device, so replays keep advancing it
    n = 1394282
    buf = torch.zeros(n, device=dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        ar(buf)
    for it in range(10):
        xs, ref = inputs(n, world, 200 + it, dev)
        buf.copy_(xs[rank])
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(buf, ref), (rank, "graph", it)
        res["checks"] += 1
    ar.check()
    # timing (kernel + launch, back-to-back on one stream)
    for label, n in (("taxi_grads_75KB", 18866), ("mnist_grads_5.58MB", 1394282), ("metrics_16B", 4)):
        for mode in modes:
            t = torch.randn(n, device=dev)
            for _ in range(20):
                ar(t, mode=mode)
            hdist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(200):
                ar(t, mode=mode)
            torch.cuda.synchronize()
            res[f"us_per_call_{label}_{mode}"] = round((time.perf_counter() - t0) / 200 * 1e6, 2)
    ar.check()
    ar.close()
    if rank == 0:
        res["ok"] = True
        print("ONESHOT " + json.dumps(res), flush=True)
    hdist.shutdown()


if __name__ == "__main__":
    main()
