"""P2P collectives (csrc/comm/oneshot.hip) failure handling and the fused data-parallel step.

* a peer that never arrives: the kernel gives up after its timeout, sets the sticky error flag and
  writes NOTHING (no sum of another epoch's staging); later launches are no-ops; poll/check raise;
* the fused DP step (reduce-scatter + sharded optimizer + all-gather) at 2 ranks sharing the GPU
  against the plain all-reduce engine (tools/dp_fused_check.py).
"""
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_p2p_timeout_writes_nothing_and_poisons():
    from hops_examples_amd.parallel import oneshot

    C = oneshot.ext()
    dev = torch.device("cuda", 0)
    # rank 0 of a 2-rank "group" whose rank 1 never launches: both staging buffers and flag pages
    # are local allocations, so only the missing peer is simulated
    n, cap = 4096, 4096
    bufs, flags = [], []
    for _ in range(2):
        b, _h = C.alloc(C.STAGING_FLOATS_PER_CAP * cap * 4, False)
        f, _h = C.alloc(C.FLAG_ROWS * C.MAX_RANKS * C.MAX_BLOCKS * 4, True)
        bufs.append(b)
        flags.append(f)
    try:
        epochs = torch.zeros(C.MAX_BLOCKS, dtype=torch.int32, device=dev)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        x = torch.ones(n, device=dev)
        out = torch.full((n,), -7.0, device=dev)
        st = torch.cuda.current_stream(dev).cuda_stream
        for two_shot in (False, True):
            C.allreduce_f32(x.data_ptr(), out.data_ptr(), n, cap, 0, 2, bufs, flags, epochs.data_ptr(),
                            err.data_ptr(), 8, st, two_shot, 0.05)
            torch.cuda.synchronize()
            assert int(err.item()) == 2  # 1 + the rank that never arrived
            assert torch.all(out == -7.0), "a timed-out reduction must not write its output"
            assert int(epochs.max().item()) == 0  # epochs not advanced
        # the fused DP step on a poisoned communicator does nothing at all
        master = torch.randn(n, device=dev)
        grad = torch.randn(n, device=dev)
        m0, g0 = master.clone(), grad.clone()
        shadow = torch.zeros(n, dtype=torch.bfloat16, device=dev)
        s1, s2 = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
        hp = torch.tensor([1.0, 0.5, 0.0, 0.95, 1e-7, 0, 0, 0], device=dev)
        step = torch.zeros(1, device=dev)
        arrive = torch.zeros(9 * 32, dtype=torch.int32, device=dev)
        C.dp_step(3, master.data_ptr(), grad.data_ptr(), s1.data_ptr(), s2.data_ptr(), 0, shadow.data_ptr(), n,
                  [1.0, 0.5, 0.0, 0.95, 1e-7], hp.data_ptr(), step.data_ptr(), arrive.data_ptr(), 0, [], [], [], 0, 0,
                  cap, 0, 2, bufs, flags, epochs.data_ptr(), err.data_ptr(), 8, st, 0.05, False, 0, [], False, [])
        torch.cuda.synchronize()
        assert torch.equal(master, m0) and torch.equal(grad, g0) and float(step.item()) == 0.0
    finally:
        for p in bufs + flags:
            C.free(p)


@pytest.mark.gpu
def test_p2p_poll_and_check_raise():
    from hops_examples_amd.parallel.oneshot import OneShotAllReduce

    ar = OneShotAllReduce(cap_bytes=1 << 16, device=torch.device("cuda", 0))  # world 1: a local sum
    x = torch.arange(1000, device="cuda", dtype=torch.float32)
    ar(x)
    ar.poll()
    ar.check()
    ar.err.fill_(3)  # as if rank 2 had never arrived
    with pytest.raises(RuntimeError, match="rank 2 never raised"):
        ar.check()
    with pytest.raises(RuntimeError, match="rank 2"):
        for _ in range(50):  # the first poll enqueues the copy; a later one reads it
            ar.poll()
            torch.cuda.synchronize()
    ar.err.zero_()
    ar.close()


# gradient paths of the fused step: zero-copy (the default: owners read the peers' arena gradients in
# place), zero-copy + per-bucket reduce-scatter during the backward (small buckets forced so the flagship
# model splits), and the staged copy
DP_MODES = {
    "zerocopy": ({}, "-zerocopy"),
    "zerocopy-overlap": ({"HOPSX_DP_MIN_SPLIT_MB": "0", "HOPSX_DP_BUCKET_MB": "1"}, "-zerocopy-overlap"),
    "copy": ({"HOPSX_P2P_ZEROCOPY": "0"}, ""),
}


@pytest.mark.gpu
@pytest.mark.parametrize("mode", sorted(DP_MODES))
def test_dp_fused_step_two_ranks(mode):
    extra, expect = DP_MODES[mode]
    env = dict(os.environ, HOPSX_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0", HOPSX_P2P="1",
               HOPSX_DPCHECK_EXPECT=expect, **extra)
    port = 29641 + sorted(DP_MODES).index(mode)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "tools", "dp_fused_check.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=110)
    assert r.returncode == 0 and "DPFUSED" in r.stdout, r.stdout[-4000:]
    print([ln for ln in r.stdout.splitlines() if "DPFUSED" in ln][-1][:600])


@pytest.mark.gpu
def test_dp_step_zero_copy_self_test_world1():
    """Zero-copy gradient paths (in place, and per-bucket reduce-scatter + pre-reduced tail) through the
    dp self-test on a world of one (the rank is its own peer), every optimizer kind."""
    from hops_examples_amd.parallel.oneshot import OneShotAllReduce, dp_self_test

    ar = OneShotAllReduce(cap_bytes=1 << 18, device=torch.device("cuda", 0))
    try:
        t = ar.make_grad_buffer(1 << 16)
        assert t is not None and ar.zero_copy and t.is_cuda and t.dtype == torch.float32
        assert int(torch.count_nonzero(t)) == 0
        assert dp_self_test(ar, rounds=6)
        assert int(torch.count_nonzero(t)) == 0  # restored (zero at rest)
    finally:
        ar.close()


@pytest.mark.gpu
@pytest.mark.parametrize("grad_bf16,weight_bf16", [(False, False), (False, True), (True, False), (True, True)])
def test_dp_step_self_test_every_wire_format(grad_bf16, weight_bf16):
    """The fused step's arithmetic in every wire format (world 1: the rank is its own peer) against
    the single-rank optimizer kernel, every optimizer kind the self-test covers, 3 rounds each."""
    from hops_examples_amd.parallel.oneshot import OneShotAllReduce, dp_self_test

    ar = OneShotAllReduce(cap_bytes=1 << 18, device=torch.device("cuda", 0))
    ar.grad_bf16, ar.weight_bf16 = grad_bf16, weight_bf16
    try:
        assert dp_self_test(ar)
        assert ar.wire_bytes_per_param(1.0) == (2 if grad_bf16 else 4) + (2 if weight_bf16 else 4)
    finally:
        ar.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["pg", "p2p"])
def test_dp_resnet_overlap_two_ranks(mode):
    """ResNet-20 (padded 8-channel stem, BN, shortcuts) on 2 ranks with the gradient exchange overlapped
    with the backward — process-group bucket all-reduces from grad_ready (pg) or the fused zero-copy
    step's per-bucket reduce-scatters (p2p) — keeps the replicas bit-identical (tools/dp_resnet_check.py)."""
    env = dict(os.environ, HOPSX_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0", HOPSX_DPR_MODE=mode)
    port = 29651 + (mode == "p2p")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "tools", "dp_resnet_check.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=110)
    assert r.returncode == 0 and "DPRESNET" in r.stdout, r.stdout[-4000:]
    print([ln for ln in r.stdout.splitlines() if "DPRESNET" in ln][-1][:400])
