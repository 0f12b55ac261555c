"""Fused last hidden Dense + classifier head (loss.hip mlp_head_k): the pre-head Dense layer's
forward is deferred into the loss kernel together with the logits layer.  Checked against the
unfused path (split-K Dense forward + head_ce) on the flagship model, gradients of every parameter
and the loss, plus a direct kernel check against an fp32 PyTorch reference."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _grads(prehead: bool):
    from hops_examples_amd import optim
    from hops_examples_amd.models.mnist import MirroredMnistCNN
    from hops_examples_amd.runtime.arena import ParamArena
    from hops_examples_amd.runtime.step import TrainStep

    os.environ["HOPSX_DEFER_PREHEAD"] = "1" if prehead else "0"
    try:
        dev = torch.device("cuda", 0)
        torch.manual_seed(3)
        m = MirroredMnistCNN().to(dev)
        for mod in m.modules():  # the same dropout masks in both runs
            if hasattr(mod, "salt"):
                mod.salt = 12345
        a = ParamArena.from_module(m, dev)
        opt = optim.Adadelta(m, lr=1.0)
        st = TrainStep(m, opt, "sparse_ce", graph=False)
        g = torch.Generator(device="cpu").manual_seed(5)
        x = torch.randint(0, 256, (32, 28, 28, 1), dtype=torch.uint8, generator=g).to(dev)
        y = torch.randint(0, 10, (32,), generator=g).to(dev)
        st._fwd_bwd(x, y)  # probe step
        a.grad.zero_()
        r = st._fwd_bwd(x, y)  # deferred step
        torch.cuda.synchronize()
        return float(r["loss"].reshape(-1)[0]), a.grad.clone(), st._prehead_w is not None
    finally:
        os.environ.pop("HOPSX_DEFER_PREHEAD", None)


def test_prehead_fusion_matches_unfused_gradients():
    la, ga, on = _grads(True)
    lb, gb, off = _grads(False)
    assert on and not off
    assert abs(la - lb) <= 1e-3 * max(1.0, abs(lb)), (la, lb)
    rel = float((ga - gb).norm() / gb.norm())
    assert rel < 1e-2, rel


def test_mlp_head_kernel_vs_fp32_reference():
    from hops_examples_amd.ops import kernels as K

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for B, Kd, N1, C in ((32, 10816, 128, 10), (17, 784, 64, 10), (8, 200, 48, 3)):
        x = torch.randn(B, Kd, device=dev).to(torch.bfloat16)
        w1 = (torch.randn(N1, Kd, device=dev) / Kd ** 0.5).to(torch.bfloat16)
        b1 = torch.randn(N1, device=dev) * 0.1
        w2 = (torch.randn(C, N1, device=dev) / N1 ** 0.5).to(torch.bfloat16)
        b2 = torch.randn(C, device=dev) * 0.1
        t = torch.randint(0, C, (B,), device=dev)
        y = torch.empty(B, N1, device=dev, dtype=torch.bfloat16)
        logits = torch.empty(B, C, device=dev, dtype=torch.bfloat16)
        dw2 = torch.zeros(C, N1, device=dev)
        db2 = torch.zeros(C, device=dev)
        loss, corr = torch.empty(1, device=dev), torch.empty(1, device=dev, dtype=torch.int32)
        for _ in range(2):  # twice: the workspace must be back at zero after a launch
            dw2.zero_()
            db2.zero_()
            dh = K.mlp_head(x, w1, b1, "relu", y, 0, logits, t, w2, b2, dw2, db2, 1.0 / B, loss, corr)
            assert dh is not False
            torch.cuda.synchronize()
        # fp32 reference
        yr = torch.relu(x.float() @ w1.float().t() + b1)
        assert torch.allclose(y.float(), yr, rtol=2e-2, atol=2e-2), float((y.float() - yr).abs().max())
        yb = y.float()  # the head sees the stored bf16 activations
        lg = yb @ w2.float().t() + b2
        lr = torch.nn.functional.cross_entropy(lg, t)
        assert abs(float(loss.item()) - float(lr)) < 2e-2 * max(1.0, float(lr)), (float(loss.item()), float(lr))
        p = torch.softmax(lg, 1)
        p[torch.arange(B), t] -= 1
        p /= B
        assert torch.allclose(dw2, p.t() @ yb, rtol=2e-2, atol=2e-3)
        assert torch.allclose(db2, p.sum(0), rtol=2e-2, atol=2e-3)
        assert torch.allclose(dh.float(), p @ w2.float(), rtol=3e-2, atol=3e-3)
