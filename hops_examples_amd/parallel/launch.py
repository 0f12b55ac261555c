"""Single-node rank launcher: ``python script.py --gpus N`` starts its own N ranks.

The driver (and a user) may run a benchmark as ``python bench.py --gpus 8`` without torchrun.  A
process that finds no ``WORLD_SIZE`` in its environment and is asked for N > 1 ranks becomes the
launcher: it never touches the GPU (``torch.cuda.device_count()`` does not initialise HIP on ROCm),
spawns N children of the same script with the torchrun environment contract (RANK / LOCAL_RANK /
WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT), forwards their output, and exits with
the first failing child's code after killing the rest — no rank is left blocked in a collective.

This is the process-per-GPU replacement of ``experiment.mirrored``'s executor reservation
(reference: notebooks/ml/Distributed_Training/mirrored_strategy/mirroredstrategy_mnist_example.ipynb:125-131,
global batch = 32 x num_replicas_in_sync).

``rehearse=True`` allows more ranks than visible GPUs: the ranks share the devices (GPU box with
one MI355X) or run on the CPU, and the process group is gloo (RCCL refuses two ranks per device).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def is_rank_process() -> bool:
    """True when a launcher (torchrun or ours) already set the rank environment."""
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def rank_exit(code: int = 0) -> None:
    """End a rank of OUR self-launch (``launch``).  By default the rank returns and exits through normal
    interpreter teardown.  Round 3 once saw a finished rehearsal rank abort in teardown ("terminate
    called without an active exception", exit -6) and made ``os._exit`` the default; the round-4
    rehearsals at 2 and 4 ranks through normal teardown exit 0 with no abort
    (profiles/r4_rehearsal_teardown.txt), so the fast exit is now opt-in: ``HOPSX_RANK_FAST_EXIT=1``
    flushes the streams and ``os._exit``s.  A no-op for ranks of other launchers (torchrun) and for
    single-process runs."""
    if os.environ.get("HOPSX_SELF_LAUNCHED") != "1" or os.environ.get("HOPSX_RANK_FAST_EXIT", "0") != "1":
        return
    try:
        sys.stdout.flush()
        sys.stderr.flush()
    finally:
        os._exit(code)


def visible_gpus() -> int:
    try:
        import torch

        return int(torch.cuda.device_count())  # does not initialise the GPU on this ROCm build
    except Exception:  # noqa: BLE001
        return 0


def _kill(procs) -> None:
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
    deadline = time.time() + 10
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.time()))
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
            p.wait()


class _Terminated(Exception):
    def __init__(self, signum: int):
        super().__init__(signum)
        self.signum = signum


def _raise_terminated(signum, frame):  # noqa: ARG001
    raise _Terminated(signum)


def _pdeathsig_setup():
    """A preexec function for each rank: die with the launcher (PR_SET_PDEATHSIG = SIGTERM), so a
    launcher killed by SIGKILL leaves no rank spinning on the GPU in its own session.  libc and prctl are
    resolved HERE, in the parent: the forked child (before exec) only calls the bound function — an
    import in the child could deadlock on a lock another parent thread (torch, a pool) held at fork.
    The child also checks that the launcher did not die before prctl took effect."""
    try:
        import ctypes

        prctl = ctypes.CDLL("libc.so.6", use_errno=True).prctl
        getppid, kill, parent = os.getppid, os.kill, os.getpid()
        sigterm, sigkill = int(signal.SIGTERM), signal.SIGKILL
    except Exception:  # noqa: BLE001
        return None

    def setup():
        prctl(1, sigterm, 0, 0, 0)
        if getppid() != parent:  # the launcher is already gone
            kill(os.getpid(), sigkill)

    return setup


def launch(nproc: int, argv: list[str], rehearse: bool = False, timeout_s: float | None = None,
           extra_env: dict | None = None) -> int:
    """Run ``sys.executable argv`` as ``nproc`` ranks on this node; returns the job's exit code.

    Refuses (returns 2, message on stderr) when fewer than ``nproc`` GPUs are visible and
    ``rehearse`` is off: a silently smaller world would report a wrong ``n_gpus``."""
    ngpu = visible_gpus()
    if ngpu < nproc and not rehearse:
        print(f"[launch] {nproc} ranks requested but {ngpu} GPU(s) visible; refusing "
              "(pass --rehearse to share devices / run on CPU with gloo)", file=sys.stderr, flush=True)
        return 2
    port = free_port()
    procs = []
    preexec = _pdeathsig_setup()
    t0 = time.time()
    rc = 0
    # a driver timeout / job manager stops the launcher with SIGTERM or SIGHUP: turn both into an
    # exception so the finally block below kills every rank (they run in sessions of their own).  Signal
    # handlers can only be installed from the main thread; elsewhere the caller's handling stands.
    import threading

    prev = {}
    try:
        if threading.current_thread() is threading.main_thread():
            prev = {sig: signal.signal(sig, _raise_terminated) for sig in (signal.SIGTERM, signal.SIGHUP)}
        for r in range(nproc):
            env = dict(os.environ)
            env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(nproc),
                        "LOCAL_WORLD_SIZE": str(nproc), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                        "MASTER_PORT": str(port), "HSA_ENABLE_IPC_MODE_LEGACY": "0", "PYTHONUNBUFFERED": "1",
                        "HOPSX_SELF_LAUNCHED": "1"})
            if rehearse and ngpu < nproc:
                env.setdefault("HOPSX_DIST_BACKEND", "gloo")
            if extra_env:
                env.update({k: str(v) for k, v in extra_env.items()})
            procs.append(subprocess.Popen([sys.executable] + list(argv), env=env, start_new_session=True,
                                          preexec_fn=preexec))
        t0 = time.time()
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0] if bad[0] > 0 else 128 - bad[0]
                print(f"[launch] a rank exited with {bad[0]}; stopping the other ranks", file=sys.stderr, flush=True)
                break
            if all(c == 0 for c in codes):
                break
            if timeout_s is not None and time.time() - t0 > timeout_s:
                print(f"[launch] job exceeded {timeout_s:g} s; stopping every rank", file=sys.stderr, flush=True)
                rc = 124
                break
            time.sleep(0.05)
    except KeyboardInterrupt:
        rc = 130
    except _Terminated as e:
        print(f"[launch] received signal {e.signum}; stopping every rank", file=sys.stderr, flush=True)
        rc = 128 + e.signum
    finally:
        _kill(procs)
        for sig, h in prev.items():
            signal.signal(sig, h)
    return rc


def rank_info(dev) -> dict:
    """What this rank sees: its place in the group and the physical device it drives."""
    import torch

    from . import dist as hdist

    info = {"rank": hdist.rank(), "world": hdist.world_size(), "device": str(dev)}
    if dev.type == "cuda":
        p = torch.cuda.get_device_properties(dev)
        info["pci"] = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
    return info


def gather_rank_info(dev, extra: dict | None = None) -> list[dict]:
    """Collective: every rank's ``rank_info`` (+ ``extra``), on every rank."""
    import torch.distributed as dist

    from . import dist as hdist

    me = rank_info(dev)
    if extra:
        me.update(extra)
    if not hdist.is_dist():
        return [me]
    out = [None] * hdist.world_size()
    dist.all_gather_object(out, me)
    return out
