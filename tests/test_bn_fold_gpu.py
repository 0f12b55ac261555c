"""BatchNorm forward apply folded into the consuming conv's operand gather (conv_mfma.hip InBn,
conv.hip hopsx_conv2d_fwd_bnstats_inbn, functional.batch_norm fold_next): against the unfused chain
bn_fwd_apply_fin -> conv2d_fwd_bnstats on the same statistics (bit-identical BN output, conv output, mean /
rstd / running statistics), and whole ResNet blocks fused vs unfused."""
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


def _acc_clean():
    for key, t in K._BN_ACC.items():
        C = (t.numel() - 12 * 32) // (2 * K.BN_NREP)
        assert int(torch.count_nonzero(t[: K.BN_NREP * 2 * C])) == 0, ("stale BN sums left in an accumulator", key)


def _load_stats(z2):
    """Put z's column sums into bn_acc(C) as a producing conv's epilogue would (replica 0 only)."""
    C = z2.shape[1]
    acc = K.bn_acc(z2.device, C)  # (the wrappers key the buffers by z.device: "cuda:0")
    acc[: K.BN_NREP * 2 * C].zero_()
    zf = z2.float()
    acc[:C] = zf.sum(0)
    acc[C:2 * C] = (zf * zf).sum(0)


# (B, H, W, C, CO, k): the ResNet-20 stage-1 / stage-2 block convs, an odd spatial size, a 16 -> 32 conv
@pytest.mark.parametrize("shape", [(8, 32, 32, 16, 16, 3), (8, 16, 16, 32, 32, 3), (3, 7, 9, 16, 16, 3),
                                   (4, 12, 10, 16, 32, 3), (4, 8, 8, 32, 16, 1)])
def test_inbn_conv_matches_apply_then_conv(shape):
    B, H, W, C, CO, k = shape
    torch.manual_seed(3)
    g = K.conv_geom((B, H, W, C), (CO, k, k, C), (1, 1), (k // 2, k // 2), (1, 1))
    z2 = bf(torch.randn(B * H * W, C, device=dev) * 1.7 + 0.4)
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.randn(C, device=dev) * 0.5
    w = bf(torch.randn(CO, k, k, C, device=dev) / (k * k * C) ** 0.5)
    res = {}
    for mode in ("apply", "fold"):
        mean, rstd = torch.empty(C, device=dev), torch.empty(C, device=dev)
        rm, rv = torch.full((C,), 0.1, device=dev), torch.full((C,), 0.9, device=dev)
        fold = (gamma, beta, mean, rstd, rm, rv, 0.1, 1e-5, "relu")
        _load_stats(z2)
        a = torch.empty(B, H, W, C, device=dev, dtype=torch.bfloat16)
        if mode == "fold":
            out = K.conv2d_fwd_bnstats_inbn(z2, a, w, g, fold)
            assert out is not None, "shape should take the folded path"
            alt = True
        else:
            K.bn_fwd_apply_fin(z2, gamma, beta, mean, rstd, rm, rv, 0.1, 1e-5, act="relu", out=a.view(-1, C))
            out = K.conv2d_fwd_bnstats(a, w, g)
            assert out is not None
            alt = False
        # consume (and re-zero) the output's statistics with its BN apply, from the buffer they went to
        o2 = out.view(-1, CO)
        m2, r2 = torch.empty(CO, device=dev), torch.empty(CO, device=dev)
        y = K.bn_fwd_apply_fin(o2, None, None, m2, r2, None, None, 0.1, 1e-5, act=0, alt=alt)
        torch.cuda.synchronize()
        res[mode] = (a.clone(), out.clone(), mean.clone(), rstd.clone(), rm.clone(), rv.clone(), m2, r2, y)
    _acc_clean()
    f, p = res["fold"], res["apply"]
    for i, name in enumerate(("bn output", "conv output", "mean", "rstd", "running mean", "running var")):
        assert torch.equal(f[i], p[i]), name
    # the output's statistics: same values, float-atomic order only
    torch.testing.assert_close(f[6], p[6], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(f[7], p[7], rtol=1e-3, atol=1e-3)
    # against fp32: act(bn(z)) and the conv
    zf = z2.float()
    ar = F.batch_norm(zf, None, None, gamma, beta, True, 0.0, 1e-5).relu()
    torch.testing.assert_close(f[0].float().view(-1, C), ar, rtol=1e-2, atol=1e-2)
    yr = F.conv2d(f[0].float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None, 1, k // 2)
    torch.testing.assert_close(f[1].float(), yr.permute(0, 2, 3, 1), rtol=2e-2, atol=2e-2)


def _blocks_step(disable, cin, cout, stride, hw, calls):
    from torch import nn

    from hops_examples_amd.models.resnet import BasicBlock

    old = os.environ.get("HOPSX_DISABLE", "")
    os.environ["HOPSX_DISABLE"] = disable
    real = K.conv2d_fwd_bnstats_inbn
    n = [0]

    def counting(*a, **kw):
        r = real(*a, **kw)
        n[0] += r is not None
        return r

    K.conv2d_fwd_bnstats_inbn = counting
    try:
        torch.manual_seed(5)
        m = nn.Sequential(BasicBlock(cin, cout, stride), BasicBlock(cout, cout)).to(dev).train()
        x = bf(torch.randn(8, hw, hw, cin, device=dev)).requires_grad_(True)
        dy = bf(torch.randn(8, hw // stride, hw // stride, cout, device=dev))
        y = m(x)
        gs = torch.autograd.grad(y, [x] + list(m.parameters()), dy)
        torch.cuda.synchronize()
        calls.append(n[0])
        stats = torch.cat([b.float().reshape(-1) for b in m.buffers()])
        return y.detach().float(), [t.float().reshape(-1) for t in gs], stats
    finally:
        K.conv2d_fwd_bnstats_inbn = real
        os.environ["HOPSX_DISABLE"] = old


@pytest.mark.parametrize("cin,cout,stride,hw", [(16, 16, 1, 32), (16, 32, 2, 32), (32, 32, 1, 16), (32, 64, 2, 16)])
def test_basic_blocks_folded_match_unfused(cin, cout, stride, hw, monkeypatch):
    """Two BasicBlocks (identity or projection first): every block's a-BN is applied inside b's conv where b's
    conv has the direct MFMA forward (9 * cout <= 512; the width gate lowered to 16 to cover that stage too);
    outputs, gradients and running statistics match the unfused step (float-atomic orders only), no statistics
    are left behind."""
    from hops_examples_amd.models.resnet import BasicBlock

    monkeypatch.setattr(BasicBlock, "fold_min_width", 16)
    calls = []
    y1, g1, s1 = _blocks_step("", cin, cout, stride, hw, calls)
    y0, g0, s0 = _blocks_step("bn_fold", cin, cout, stride, hw, calls)
    _acc_clean()
    assert calls == ([2, 0] if 9 * cout <= 512 else [0, 0]), calls
    torch.testing.assert_close(y1, y0, rtol=3e-2, atol=3e-2)
    assert float(F.cosine_similarity(y1.reshape(-1), y0.reshape(-1), dim=0)) > 0.9999
    torch.testing.assert_close(s1, s0, rtol=1e-3, atol=1e-3)
    rel = [float((u - v).norm() / v.norm().clamp_min(1e-12)) for u, v in zip(g1, g0)]
    cos = float(F.cosine_similarity(torch.cat(g1), torch.cat(g0), dim=0))
    assert cos > 0.999 and max(rel) < 0.05, (cos, rel)


def test_fold_falls_back_to_apply_without_the_path():
    """A fold_next BN whose consumer conv has no folded path (K = 9 * 64 > 512) is applied by its own launch
    just before the conv: same result as without fold_next."""
    from hops_examples_amd.models.resnet import ConvBN

    outs = []
    for fold in (True, False):
        torch.manual_seed(9)
        a, b = ConvBN(64, 64, 3).to(dev).train(), ConvBN(64, 64, 3).to(dev).train()
        x = bf(torch.randn(4, 8, 8, 64, device=dev))
        outs.append(b(a(x, fold_next=fold)).float())
    torch.cuda.synchronize()
    _acc_clean()
    torch.testing.assert_close(outs[0], outs[1], rtol=2e-2, atol=2e-2)


def test_resnet20_per_layer_with_folded_bn_vs_fp64():
    """ResNet-20 with the a-BNs of the 16 / 32-channel stages applied inside the b convs: every op's output
    and every parameter gradient against the teacher-forced bf16-emulating fp64 reference (runtime/layercheck)."""
    from hops_examples_amd.runtime import layercheck as LC

    real, n = K.conv2d_fwd_bnstats_inbn, [0]

    def counting(*a, **kw):
        r = real(*a, **kw)
        n[0] += r is not None
        return r

    K.conv2d_fwd_bnstats_inbn = counting
    try:
        r = LC.resnet20_check(32, "")
    finally:
        K.conv2d_fwd_bnstats_inbn = real
    _acc_clean()
    # the 32-channel stage's 3 blocks (the 16-channel stage is below BasicBlock.fold_min_width; the 64-channel
    # stage has K = 576: no direct MFMA forward)
    assert n[0] == 3, n[0]
    assert r["min_grad_cos"] > 0.999 and r["min_fwd_cos"] > 0.9999, (r["min_grad_cos"], r["min_fwd_cos"])
