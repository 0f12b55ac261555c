"""A passive peer PROCESS for the persistent flagship's data-parallel exchange (cross-process test).

The active process runs the real DP kernel as rank q of W (runtime/persist_sim.py ExchangeSim, peers
pointed at THIS process's buffers).  This process:

  1. allocates its own uncached exchange buffer and flag page and hands their IPC handles over;
  2. maps the active rank's buffer and flag page from the handles it receives;
  3. on "go" — while the active kernel is already spinning on its flag page — pushes the other ranks'
     payloads into the active rank's buffer with system-scope stores (``xpush``), then raises every
     flag word of the active rank's page to the step's epoch in a second launch (``xfill``): the
     producer half of the hand-off, from another process, through IPC mappings of uncached memory;
  4. on "check" compares what the active kernel pushed into THIS process's buffer (slot q) with the
     payload the single-process run harvested for rank q — the active kernel's producer half.

Protocol: one JSON object per line on stdin / stdout.  Run as
``python -m hops_examples_amd.runtime.persist_peer``; the test drives it
(tests/test_persist_dp_sim_gpu.py::test_cross_process_peer).
"""
from __future__ import annotations

import json
import sys
import time


def _out(obj) -> None:
    sys.stdout.write(json.dumps(obj) + "\n")
    sys.stdout.flush()


def _in() -> dict:
    line = sys.stdin.readline()
    if not line:
        raise SystemExit(3)
    return json.loads(line)


def main() -> int:
    import torch

    from ..parallel import oneshot
    from .persist import geometry
    from .persist_sim import REGIONS

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    C = oneshot.ext()
    g = geometry()
    buf, hb = C.alloc(int(g["x_bytes"]), True)
    flg, hf = C.alloc(int(g["xflag_words"]) * 4, True)
    _out({"hb": bytes(hb).hex(), "hf": bytes(hf).hex()})
    msg = _in()
    abuf = C.open(bytes.fromhex(msg["hb"]))
    aflg = C.open(bytes.fromhex(msg["hf"]))
    q = int(msg["rank"])
    pay = torch.load(msg["payload"], weights_only=True)
    peers = {int(r): {n: t.to(dev) for n, t in regs.items()} for r, regs in pay["peers"].items()}
    expect = {n: t.to(dev) for n, t in pay["expect"].items()}

    def region(base, name, slot):
        xo, xs = int(g["xo_" + name]), int(g["xs_" + name])
        return base + xo + slot * xs, xs  # parity 0

    torch.cuda.synchronize()
    _out({"ready": 1})
    msg = _in()
    time.sleep(float(msg.get("delay_ms", 20)) / 1000.0)  # the active kernel is spinning by now
    st = torch.cuda.current_stream().cuda_stream
    for r, regs in peers.items():
        for n in REGIONS:
            ptr, nb = region(abuf, n, r)
            C.xpush(ptr, regs[n].data_ptr(), nb, st)
    C.xfill(aflg, int(g["xflag_words"]), int(msg["go"]) & 0xFFFFFFFF, st)
    torch.cuda.synchronize()
    _out({"pushed": 1})
    _in()  # "check": the active kernel has finished
    match, diffs = True, {}
    for n in REGIONS:
        ptr, nb = region(buf, n, q)
        t = torch.empty(nb, dtype=torch.uint8, device=dev)
        C.copy(t.data_ptr(), ptr, nb)
        d = int((t != expect[n]).sum())
        diffs[n] = d
        match = match and d == 0
    _out({"match": match, "diffs": diffs})
    torch.cuda.synchronize()
    C.close(abuf)
    C.close(aflg)
    C.free(buf)
    C.free(flg)
    return 0


if __name__ == "__main__":
    sys.exit(main())
