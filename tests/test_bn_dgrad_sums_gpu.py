"""BatchNorm backward column sums reduced in the consumer conv's dgrad epilogue (conv_mfma.hip DgradArgs
bnacc) + the apply-only BN backward (norm.hip hopsx_bn_bwd_pre), against the unfused chain: the plain
paired conv backward, then the full BN backward (bn_colred8_k + bn_bwd_apply_fin8_k)."""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd.ops import functional as HF  # noqa: E402
from hops_examples_amd.ops import kernels as K  # noqa: E402

dev = "cuda"


def bf(t):
    return t.to(torch.bfloat16)


def _acc_clean():
    for t in K._BN_ACC.values():
        C = (t.numel() - 12 * 32) // (2 * K.BN_NREP)
        assert int(torch.count_nonzero(t[: K.BN_NREP * 2 * C])) == 0, "stale BN sums left in an accumulator"


# (B, H, W, C = the BN width = conv input channels, CO, k): ResNet-20 stage-1 / stage-2 shapes (direct MFMA
# dgrad), stage 3 (K = 576: the implicit-GEMM dgrad with EpiDgradBnBF16)
@pytest.mark.parametrize("shape", [(8, 32, 32, 16, 16, 3), (8, 16, 16, 32, 32, 3), (3, 7, 9, 32, 32, 3),
                                   (8, 8, 8, 64, 64, 3)])
@pytest.mark.parametrize("with_addend", [False, True])
def test_pair_bn_sums_match_unfused(shape, with_addend):
    B, H, W, C, CO, k = shape
    torch.manual_seed(7)
    g = K.conv_geom((B, H, W, C), (CO, k, k, C), (1, 1), (k // 2, k // 2), (1, 1))
    assert K.conv2d_bwd_pair_bn_ok(g)
    z = bf(torch.randn(B * H * W, C, device=dev) * 2 + 0.3)  # the BN input
    zf = z.float()
    mean = zf.mean(0)
    rstd = (zf.var(0, unbiased=False) + 1e-5).rsqrt()
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.randn(C, device=dev) * 0.5
    x = bf(((zf - mean) * rstd * gamma + beta).relu()).view(B, H, W, C)  # BN + ReLU output = conv input
    w = bf(torch.randn(CO, k, k, C, device=dev) / (k * k * C) ** 0.5)
    dy = bf(torch.randn(B, H, W, CO, device=dev))
    add = bf(torch.randn(B, H, W, C, device=dev)) if with_addend else None
    res = {}
    for mode in ("plain", "bn"):
        dw = torch.zeros(CO, k, k, C, device=dev)
        gg, gb, ws = torch.zeros(C, device=dev), torch.zeros(C, device=dev), torch.empty(2 * C, device=dev)
        if mode == "bn":
            dX = K.conv2d_bwd_pair(dy, w, g, x, dw, addend=add, bn=(z, mean, rstd, x, "relu"))
            assert dX is not False
            dz = K.bn_bwd_pre(dX.view(-1, C), z, gamma, mean, rstd, gg, gb, ws)
        else:
            dX = K.conv2d_bwd_pair(dy, w, g, x, dw, addend=add)
            assert dX is not False
            dz = K.bn_bwd(dX.view(-1, C), z, x.view(-1, C), gamma, mean, rstd, gg, gb, ws, act="relu")
            dX = dX * (x > 0)  # the bn path stores the masked gradient
        res[mode] = (dX.float(), dz.float(), gg.clone(), gb.clone(), dw.clone())
    torch.cuda.synchronize()
    _acc_clean()
    p, b = res["plain"], res["bn"]
    assert torch.equal(b[0], p[0]), "masked dX must be bit-identical"
    torch.testing.assert_close(b[4], p[4], rtol=1e-3, atol=1e-3)  # weight gradient (float-atomic order only)
    torch.testing.assert_close(b[2], p[2], rtol=1e-3, atol=1e-2)  # dgamma = sum g * xhat
    torch.testing.assert_close(b[3], p[3], rtol=1e-3, atol=1e-2)  # dbeta = sum g
    torch.testing.assert_close(b[1], p[1], rtol=2e-2, atol=2e-2)
    # against fp32 autograd of the BN + ReLU on the same masked gradient
    zr = zf.clone().requires_grad_(True)
    yr = F.batch_norm(zr, None, None, gamma, beta, True, 0.0, 1e-5).relu()
    yr.backward(p[0].view(-1, C))
    torch.testing.assert_close(b[1], zr.grad, rtol=3e-2, atol=3e-2)


def _resnet_step(disable: str, calls: list | None = None):
    from hops_examples_amd.models.resnet import cifar_resnet

    old = os.environ.get("HOPSX_DISABLE", "")
    os.environ["HOPSX_DISABLE"] = disable
    real = K.bn_bwd_pre
    n = [0]

    def counting(*a, **kw):
        n[0] += 1
        return real(*a, **kw)

    K.bn_bwd_pre = counting
    try:
        torch.manual_seed(0)
        m = cifar_resnet(20).to(dev).train()
        x = torch.randint(0, 256, (32, 32, 32, 3), device=dev, dtype=torch.uint8)
        y = torch.randint(0, 10, (32,), device=dev)
        logits = m(x)
        F.cross_entropy(logits.float(), y).backward()
        torch.cuda.synchronize()
        grads = torch.cat([p.grad.float().reshape(-1) for p in m.parameters() if p.grad is not None])
        if calls is not None:
            calls.append(n[0])
        return grads
    finally:
        K.bn_bwd_pre = real
        os.environ["HOPSX_DISABLE"] = old


def test_resnet20_step_with_bn_sums_in_dgrad():
    """ResNet-20: every BN whose output feeds a paired-backward conv as its only consumer (all but the two
    BNs in front of projection blocks and the last one) takes the fused path; gradients match the unfused
    step, no sums are left behind."""
    calls = []
    g1 = _resnet_step("", calls)
    g1b = _resnet_step("")
    g0 = _resnet_step("bn_dgrad_sums", calls)
    _acc_clean()
    assert not HF._BNPRE, "a reduced gradient was never consumed by its BN"
    assert calls[0] >= 15 and calls[1] == 0, calls
    noise = float(F.cosine_similarity(g1b, g1, dim=0))
    cos = float(F.cosine_similarity(g1, g0, dim=0))
    assert cos > 0.99 and cos > noise - 0.01, (cos, noise)
