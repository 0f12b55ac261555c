"""Conv forward with the BatchNorm statistics in its epilogue (conv_mfma.hip BNS / conv.hip
EpiBnStatsBF16) + the one-launch BN apply that finalizes them (norm.hip bn_apply_fin8_k), against
plain PyTorch fp32 conv -> batch_norm -> (+ residual) -> ReLU, and a whole ResNet-20 step with the
fusion on vs off."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd.ops import kernels as K  # noqa: E402

dev = "cuda"


def bf(t):
    return t.to(torch.bfloat16)


def close(a, b, rtol=2e-2, atol=2e-2):
    torch.testing.assert_close(a.float(), b.float(), rtol=rtol, atol=atol)


# (B, H, W, C, CO, k, stride): direct-MFMA path (K <= 512) and the implicit-GEMM path (K = 576)
SHAPES = [(8, 32, 32, 16, 16, 3, 1), (8, 16, 16, 32, 64, 3, 2), (8, 8, 8, 64, 64, 3, 1), (8, 32, 32, 16, 32, 1, 2),
          (4, 14, 14, 128, 128, 3, 1)]


@pytest.mark.parametrize("shape", SHAPES)
def test_conv_bnstats_then_apply(shape):
    B, H, W, C, CO, k, s = shape
    torch.manual_seed(3)
    x = bf(torch.randn(B, H, W, C, device=dev))
    w = bf(torch.randn(CO, k, k, C, device=dev) / (k * k * C) ** 0.5)
    res = bf(torch.randn(B, (H + s - 1) // s, (W + s - 1) // s, CO, device=dev))
    gamma = torch.rand(CO, device=dev) + 0.5
    beta = torch.randn(CO, device=dev)
    g = K.conv_geom(x.shape, w.shape, (s, s), (k // 2, k // 2), (1, 1))
    for rep in range(2):  # twice: the accumulator must be back at zero after the first apply
        y = K.conv2d_fwd_bnstats(x, w, g)
        assert y is not None, "shape should have the statistics epilogue"
        mean, rstd = torch.empty(CO, device=dev), torch.empty(CO, device=dev)
        rm, rv = torch.zeros(CO, device=dev), torch.ones(CO, device=dev)
        out = K.bn_fwd_apply_fin(y.view(-1, CO), gamma, beta, mean, rstd, rm, rv, 0.1, 1e-5,
                                 residual=res.view(-1, CO), act="relu")
    torch.cuda.synchronize()
    assert int(torch.count_nonzero(K.bn_acc(torch.device(dev), CO))) == 0
    yr = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None, s, k // 2)
    close(y.permute(0, 3, 1, 2), yr, rtol=1e-2, atol=1e-2)
    yb = y.float().view(-1, CO)  # statistics of the stored bf16 conv output, as the kernel sees it
    rm2, rv2 = torch.zeros(CO, device=dev), torch.ones(CO, device=dev)
    ref = (F.batch_norm(yb, rm2, rv2, gamma, beta, True, 0.1, 1e-5) + res.float().view(-1, CO)).relu()
    close(out, ref)
    close(mean, yb.mean(0), rtol=1e-3, atol=1e-4)
    close(rstd, (yb.var(0, unbiased=False) + 1e-5).rsqrt(), rtol=1e-3, atol=1e-3)
    close(rm, rm2, rtol=1e-3, atol=1e-4)
    close(rv, rv2, rtol=1e-3, atol=1e-4)


def _resnet_step(disable: str):
    from hops_examples_amd.models.resnet import cifar_resnet

    old = os.environ.get("HOPSX_DISABLE", "")
    os.environ["HOPSX_DISABLE"] = disable
    try:
        torch.manual_seed(0)
        m = cifar_resnet(20).to(dev).train()
        x = torch.randint(0, 256, (16, 32, 32, 3), device=dev, dtype=torch.uint8)
        y = torch.randint(0, 10, (16,), device=dev)
        logits = m(x)
        loss = F.cross_entropy(logits.float(), y)
        loss.backward()
        grads = torch.cat([p.grad.float().reshape(-1) for p in m.parameters() if p.grad is not None])
        bufs = torch.cat([b.float().reshape(-1) for n, b in m.named_buffers() if "running" in n])
        return logits.float().detach(), grads, bufs
    finally:
        os.environ["HOPSX_DISABLE"] = old


def test_resnet20_step_bnstats_matches_unfused():
    """Same logits / running statistics; the one-step gradients agree to cos > 0.97.

    Why not tighter (profiles/r4_bn_gap_resnet20.txt, tools/bn_gap.py, deterministic mode so both
    paths are bit-reproducible): the two paths sum the BN statistics in a different order (conv
    epilogue per-tile partials vs the statistics pass), so a mean / rstd differs in the last bit.
    The stem and block-0 convs/BNs come out bit-identical; the first difference is 6e-6 at
    blocks.0.b.bn, and this random-init ResNet-20 then roughly doubles it every layer (1.5e-2 at
    the last block) and the backward takes the gradient to ~0.19 relative (cos 0.989).  Any equally
    valid reordering (another GEMM tiling) does the same: it is the network's sensitivity at init,
    not a defect of either path — the single ConvBN layer test below is the tight comparison."""
    l0, g0, b0 = _resnet_step("bnstats")
    _, g0b, _ = _resnet_step("bnstats")
    l1, g1, b1 = _resnet_step("")
    close(l1, l0, rtol=3e-2, atol=3e-2)
    close(b1, b0, rtol=1e-2, atol=1e-2)
    noise = float(F.cosine_similarity(g0b, g0, dim=0))
    cos = float(F.cosine_similarity(g1, g0, dim=0))
    assert cos > 0.97 and cos > noise - 0.02, (cos, noise)  # measured: cos 0.989 .. 0.995, noise ~1


def test_convbn_layer_grads_bnstats_matches_unfused():
    """One ConvBN (+ residual + ReLU) layer: forward and all gradients, fused vs unfused."""
    from hops_examples_amd.models.resnet import ConvBN

    out = {}
    for dis in ("bnstats", ""):
        old = os.environ.get("HOPSX_DISABLE", "")
        os.environ["HOPSX_DISABLE"] = dis
        try:
            torch.manual_seed(1)
            m = ConvBN(32, 32, 3).to(dev).train()
            x = bf(torch.randn(32, 16, 16, 32, device=dev)).requires_grad_(True)
            r = bf(torch.randn(32, 16, 16, 32, device=dev)).requires_grad_(True)
            y = m(x, residual=r)
            dy = bf(torch.randn_like(y.float()))
            gx, gr = torch.autograd.grad(y, (x, r), dy, retain_graph=True)
            out[dis] = (y.float(), gx.float(), gr.float())
        finally:
            os.environ["HOPSX_DISABLE"] = old
    for a, b in zip(out[""], out["bnstats"]):
        close(a, b, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("C,H", [(16, 16), (32, 8), (64, 8)])
def test_identity_block_residual_grad_in_dgrad_epilogue(C, H):
    """BasicBlock with an identity shortcut: the residual's gradient handed to conv a's dgrad
    (epilogue addend on the direct MFMA pair, a separate add on the GEMM variant) equals autograd's
    accumulation of the two parts (HOPSX_DISABLE=res_addend)."""
    from hops_examples_amd.models.resnet import BasicBlock

    out = {}
    for dis in ("res_addend", ""):
        old = os.environ.get("HOPSX_DISABLE", "")
        os.environ["HOPSX_DISABLE"] = dis
        try:
            torch.manual_seed(4)
            m = BasicBlock(C, C).to(dev).train()
            x = bf(torch.randn(32, H, H, C, device=dev)).requires_grad_(True)
            y = m(x)
            dy = bf(torch.randn_like(y.float()))
            gx, = torch.autograd.grad(y, (x,), dy)
            out[dis] = (y.float(), gx.float())
        finally:
            os.environ["HOPSX_DISABLE"] = old
    for a, b in zip(out[""], out["res_addend"]):
        close(a, b, rtol=2e-2, atol=2e-2)


def _resnet_fp64_reference(m, x_u8, y):
    """Plain PyTorch fp64 one-step forward/backward of a CifarResNet with the module's own fp32 master
    weights: NCHW F.conv2d / train-mode F.batch_norm / avg-pool / linear / cross-entropy, no hopsx code.
    Returns (logits, flat gradient in m.parameters() order, running stats after the step)."""
    d = torch.float64
    ps = [p.detach().to(d).clone().requires_grad_(True) for p in m.parameters()]
    P = dict(zip([n for n, _ in m.named_parameters()], ps))
    run = {n: b.detach().to(d).clone() for n, b in m.named_buffers() if "running" in n}
    x = x_u8.to(d)
    x = x * torch.tensor(m.img_scale_c, dtype=d, device=x.device) + torch.tensor(m.img_shift_c, dtype=d, device=x.device)
    x = x.permute(0, 3, 1, 2)

    def convbn(pre, mod, t, residual=None):
        w = P[pre + ".conv.weight"].permute(0, 3, 1, 2)
        t = F.conv2d(t, w, None, mod.conv.cfg["stride"], mod.conv.kernel_size[0] // 2)
        t = F.batch_norm(t, run[pre + ".bn.running_mean"], run[pre + ".bn.running_var"], P[pre + ".bn.weight"],
                         P[pre + ".bn.bias"], True, mod.bn.momentum, mod.bn.eps)
        if residual is not None:
            t = t + residual
        return t.relu() if mod.bn.activation == "relu" else t

    h = convbn("stem", m.stem, x)
    for i, blk in enumerate(m.blocks):
        pre = f"blocks.{i}"
        s = h if blk.short is None else convbn(pre + ".short", blk.short, h)
        a = convbn(pre + ".a", blk.a, h)
        h = convbn(pre + ".b", blk.b, a, residual=s)  # act(bn(conv(a)) + shortcut), as HF.batch_norm
    logits = F.linear(h.mean((2, 3)), P["fc.weight"], P["fc.bias"])
    F.cross_entropy(logits, y).backward()
    g = torch.cat([p.grad.reshape(-1) for p in ps])
    bufs = torch.cat([run[n].reshape(-1) for n, _ in m.named_buffers() if "running" in n])
    return logits.detach(), g, bufs


def test_resnet20_step_fused_and_unfused_vs_fp64():
    """Both BN-statistics paths against an fp64 PyTorch ResNet-20 step on the same weights and batch.

    Settles the fused-vs-unfused gap of test_resnet20_step_bnstats_matches_unfused: if the fused path
    (statistics in the conv epilogue) were wrong, its cosine to fp64 would sit clearly below the
    unfused path's.  Both carry the same bf16-activation error, so both cosines must be high and
    within a small margin of each other (measured values are printed)."""
    from hops_examples_amd.models.resnet import cifar_resnet

    torch.manual_seed(0)
    m = cifar_resnet(20).to(dev).train()
    x = torch.randint(0, 256, (16, 32, 32, 3), device=dev, dtype=torch.uint8)
    y = torch.randint(0, 10, (16,), device=dev)
    torch.manual_seed(0)
    lr, gr, br = _resnet_fp64_reference(m, x, y)
    res = {}
    for dis in ("bnstats", ""):
        l, g, b = _resnet_step(dis)
        res[dis or "fused"] = (float(F.cosine_similarity(g.double(), gr, dim=0)),
                               float((l.double() - lr).abs().max()), float((b.double() - br).abs().max()))
    print("fp64 cos / max|dlogit| / max|drunning|:", res)
    cf, cu = res["fused"][0], res["bnstats"][0]
    assert cf > 0.95 and cu > 0.95, res
    # the free-running fp64 step measures the random-init network's sensitivity (a last-bit difference
    # doubles per layer); the kernels themselves are held per layer, against fp64 at their own operating
    # point (runtime/layercheck.py, tests/test_resnet_layers_gpu.py: worst tensor 0.99984 measured)
    from hops_examples_amd.runtime import layercheck as LC

    for dis in ("bnstats", ""):
        r = LC.resnet20_check(16, dis)
        assert r["min_grad_cos"] > 0.999 and r["min_fwd_cos"] > 0.9999, (dis, r["min_grad_cos"], r["min_fwd_cos"])
    assert abs(cf - cu) < 0.02, res  # neither path is systematically further from fp64
    for k in res:
        assert res[k][1] < 0.1 and res[k][2] < 0.05, res
