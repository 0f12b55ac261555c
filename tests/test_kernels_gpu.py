"""Numerics of every gfx950 HIP kernel against a plain PyTorch fp32 reference.

Inputs are rounded to bf16 first, so the reference sees exactly the operands
the MFMA kernels see; tolerances then only cover fp32-accumulation order and
the final bf16 rounding of outputs.  Shapes cover every workload in
SURVEY.md §2.5 (incl. unaligned N=20/50, K=4/9/16/25, stride-2 and 7x7 stems).
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd.ops import kernels as K  # noqa: E402
from hops_examples_amd.ops import _C  # noqa: E402

dev = "cuda"


def bf(t):
    return t.to(torch.bfloat16)


def close(a, b, rtol=2e-2, atol=2e-2):
    a = a.float()
    b = b.float()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err <= atol * scale + rtol * scale or err <= atol, f"max err {err} vs scale {scale}"


def test_extension_is_native():
    m = _C.ext()
    assert m.ARCH == "gfx950"
    assert m.__file__.endswith(".so")


@pytest.mark.parametrize("M,Kd,N", [(32, 1600, 128), (32, 10816, 128), (64, 800, 500), (64, 500, 10), (1000, 784, 128),
                                    (300, 77, 50), (4096, 512, 256), (7, 13, 5), (513, 1024, 1000), (10, 6, 64)])
@pytest.mark.parametrize("act", ["none", "relu"])
def test_linear_fwd(M, Kd, N, act):
    torch.manual_seed(0)
    x = bf(torch.randn(M, Kd, device=dev))
    w = bf(torch.randn(N, Kd, device=dev) / math.sqrt(Kd))
    b = torch.randn(N, device=dev)
    y = K.linear_fwd(x, w, b, act=act)
    ref = x.float() @ w.float().t() + b
    if act == "relu":
        ref = ref.relu()
    close(y, ref)
    y32 = K.linear_fwd(x, w, b, act=act, out_f32=True)
    close(y32, ref, rtol=1e-3, atol=1e-3)


def test_linear_asymmetric_layout():
    # A = I, asymmetric B catches a transposed C-write (guide §3)
    n = 64
    x = bf(torch.eye(n, device=dev))
    w = bf(torch.arange(n * n, device=dev, dtype=torch.float32).reshape(n, n) % 17)
    y = K.linear_fwd(x, w, out_f32=True)
    assert torch.equal(y, w.float().t())


@pytest.mark.parametrize("M,Kd,N", [(32, 1600, 128), (64, 800, 500), (300, 77, 50), (2048, 256, 384), (33, 20, 10)])
def test_linear_dgrad_wgrad(M, Kd, N):
    torch.manual_seed(1)
    x = bf(torch.randn(M, Kd, device=dev)).relu()
    w = bf(torch.randn(N, Kd, device=dev) / math.sqrt(Kd))
    dy = bf(torch.randn(M, N, device=dev))
    dx = K.linear_dgrad(dy, w)
    close(dx, dy.float() @ w.float())
    cs = torch.zeros(Kd, device=dev)
    dx2 = K.linear_dgrad(dy, w, yprev=x, act_prev="relu", colsum=cs)
    ref2 = (dy.float() @ w.float()) * (x.float() > 0)
    close(dx2, ref2)
    close(cs, ref2.sum(0), rtol=3e-2, atol=3e-2)
    dw = torch.zeros(N, Kd, device=dev)
    K.linear_wgrad(dy, x, dw)
    close(dw, dy.float().t() @ x.float(), rtol=1e-2, atol=1e-2)
    K.linear_wgrad(dy, x, dw)  # accumulates
    close(dw, 2 * (dy.float().t() @ x.float()), rtol=1e-2, atol=1e-2)


CONV_CASES = [
    # B, H, W, C, CO, k, stride, pad
    (32, 28, 28, 1, 32, 2, 1, 0),     # mirrored MNIST conv1
    (32, 27, 27, 32, 64, 2, 1, 0),    # mirrored MNIST conv2
    (32, 28, 28, 1, 32, 4, 1, 0),     # keras MNIST conv1
    (32, 25, 25, 32, 64, 4, 1, 0),
    (16, 28, 28, 1, 32, 3, 1, 1),     # grid-search 'same'
    (16, 28, 28, 32, 64, 3, 1, 1),
    (64, 28, 28, 1, 20, 5, 1, 0),     # pytorch Net conv1 (N=20)
    (64, 12, 12, 20, 50, 5, 1, 0),    # pytorch Net conv2 (N=50, C=20)
    (8, 16, 16, 64, 128, 3, 2, 1),    # resnet stride-2
    (4, 32, 32, 3, 64, 7, 2, 3),      # resnet stem
    (8, 8, 8, 64, 256, 1, 1, 0),      # 1x1 bottleneck
]


@pytest.mark.parametrize("B,H,W,C,CO,k,s,p", CONV_CASES)
def test_conv2d(B, H, W, C, CO, k, s, p):
    torch.manual_seed(2)
    x = bf(torch.randn(B, H, W, C, device=dev)).relu()
    w = bf(torch.randn(CO, k, k, C, device=dev) / math.sqrt(k * k * C))
    bias = torch.randn(CO, device=dev)
    g = K.conv_geom(x.shape, w.shape, (s, s), (p, p), (1, 1))
    y = K.conv2d_fwd(x, w, g, bias=bias, act="relu")
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.conv2d(xr, wr, bias, stride=s, padding=p).relu()
    close(y, yr.permute(0, 2, 3, 1))
    dy = bf(torch.randn_like(y.float()))
    dyr = dy.float().permute(0, 3, 1, 2)
    # pre-activation gradient for the conv itself
    pre = F.conv2d(xr, wr, bias, stride=s, padding=p)
    gx, gw = torch.autograd.grad(pre, (xr, wr), dyr)
    dx = K.conv2d_dgrad(dy, w, g)
    close(dx, gx.permute(0, 2, 3, 1))
    dx2 = K.conv2d_dgrad(dy, w, g, yprev=x, act_prev="relu")
    close(dx2, gx.permute(0, 2, 3, 1) * (x.float() > 0))
    dw = torch.zeros(CO, k, k, C, device=dev)
    K.conv2d_wgrad(dy, x, g, dw)
    close(dw, gw.permute(0, 2, 3, 1), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("B,H,W,C,k,s,p", [(32, 26, 26, 64, 2, 2, 0), (32, 22, 22, 64, 4, 4, 0), (8, 16, 16, 64, 3, 2, 1)])
def test_maxpool(B, H, W, C, k, s, p):
    torch.manual_seed(3)
    x = bf(torch.randn(B, H, W, C, device=dev))
    y, am = K.maxpool2d_fwd(x, (k, k), (s, s), (p, p))
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.max_pool2d(xr, k, s, p)
    close(y, yr.permute(0, 2, 3, 1), rtol=0, atol=1e-6)
    dy = bf(torch.randn_like(y.float()))
    (gx,) = torch.autograd.grad(yr, (xr,), dy.float().permute(0, 3, 1, 2))
    cs = torch.zeros(C, device=dev)
    dx = K.maxpool2d_bwd(dy, am, x.shape, (k, k), (s, s), (p, p), colsum=cs)
    close(dx, gx.permute(0, 2, 3, 1))
    close(cs, gx.sum((0, 2, 3)), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("B,C", [(32, 10), (64, 10), (1000, 1000), (5, 130)])
def test_softmax_xent(B, C):
    torch.manual_seed(4)
    z = torch.randn(B, C, device=dev) * 3
    lab = torch.randint(0, C, (B,), device=dev)
    ls = torch.zeros(1, device=dev)
    cor = torch.zeros(1, device=dev, dtype=torch.int32)
    dl = torch.empty(B, C, device=dev)
    K.loss_fwd_bwd(0, z, lab, 1.0 / B, ls, cor, dl)
    zr = z.clone().requires_grad_(True)
    lr = F.cross_entropy(zr, lab)
    (gr,) = torch.autograd.grad(lr, (zr,))
    assert abs(ls.item() - lr.item()) < 1e-4 * max(1, abs(lr.item()))
    close(dl, gr, rtol=1e-4, atol=1e-5)
    assert cor.item() == (z.argmax(1) == lab).sum().item()
    # dense one-hot targets
    oh = F.one_hot(lab, C).float()
    ls.zero_(); cor.zero_()
    K.loss_fwd_bwd(1, z, oh, 1.0 / B, ls, cor, dl)
    assert abs(ls.item() - lr.item()) < 1e-4 * max(1, abs(lr.item()))
    close(dl, gr, rtol=1e-4, atol=1e-5)
    # bf16 logits / grads
    zb = bf(z)
    dlb = torch.empty(B, C, device=dev, dtype=torch.bfloat16)
    ls.zero_()
    K.loss_fwd_bwd(0, zb, lab, 1.0 / B, ls, cor, dlb)
    close(dlb, F.softmax(zb.float(), 1).sub(oh).div(B))


def test_bce_mse():
    torch.manual_seed(5)
    B = 257
    z = torch.randn(B, 1, device=dev)
    y = (torch.rand(B, 1, device=dev) > 0.5).float()
    ls = torch.zeros(1, device=dev)
    cor = torch.zeros(1, device=dev, dtype=torch.int32)
    dl = torch.empty_like(z)
    K.loss_fwd_bwd(2, z, y, 1.0 / B, ls, cor, dl)
    zr = z.clone().requires_grad_(True)
    l = F.binary_cross_entropy_with_logits(zr, y)
    (g,) = torch.autograd.grad(l, (zr,))
    assert abs(ls.item() - l.item()) < 1e-4
    close(dl, g, rtol=1e-4, atol=1e-6)
    ls.zero_()
    K.loss_fwd_bwd(3, z, y, 1.0 / B, ls, cor, dl)
    l = F.mse_loss(zr, y)
    (g,) = torch.autograd.grad(l, (zr,))
    assert abs(ls.item() - l.item()) < 1e-4
    close(dl, g, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("name", ["sgd", "adam", "adamw", "adadelta", "rmsprop", "rmsprop_plain", "adagrad"])
def test_optimizers(name):
    torch.manual_seed(6)
    n = 100_003
    p0 = torch.randn(n, device=dev)
    grads = [torch.randn(n, device=dev) for _ in range(3)]
    ref = p0.clone().requires_grad_(True)
    cfg = {
        "sgd": (torch.optim.SGD, dict(lr=0.1, momentum=0.9, nesterov=True, weight_decay=1e-4), [0.1, 1.0, 1e-4, 0.9, 0.0, 1.0]),
        "adam": (torch.optim.Adam, dict(lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2), [1e-3, 1.0, 1e-2, 0.9, 0.999, 1e-8]),
        "adamw": (torch.optim.AdamW, dict(lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2), [1e-3, 1.0, 1e-2, 0.9, 0.999, 1e-8]),
        "adadelta": (torch.optim.Adadelta, dict(lr=1.0, rho=0.95, eps=1e-7), [1.0, 1.0, 0.0, 0.95, 1e-7]),
        "rmsprop": (torch.optim.RMSprop, dict(lr=0.01, alpha=0.9, eps=1e-7, momentum=0.5, centered=True), [0.01, 1.0, 0.0, 0.9, 1e-7, 0.5, 1.0]),
        # no momentum, not centered: the kernel skips the two unused state streams (optim.hip s23)
        "rmsprop_plain": (torch.optim.RMSprop, dict(lr=0.01, alpha=0.9, eps=1e-7), [0.01, 1.0, 0.0, 0.9, 1e-7, 0.0, 0.0]),
        "adagrad": (torch.optim.Adagrad, dict(lr=0.1, eps=1e-10), [0.1, 1.0, 0.0, 1e-10]),
    }[name]
    opt = cfg[0]([ref], **cfg[1])
    p = p0.clone()
    s1, s2, s3 = (torch.zeros(n, device=dev) for _ in range(3))
    shadow = torch.empty(n, device=dev, dtype=torch.bfloat16)
    step = torch.zeros(1, device=dev)
    for g in grads:
        ref.grad = g.clone()
        opt.step()
        gg = g.clone()
        K.optim_step(_C.OPTIM[name.replace("_plain", "")], p, gg, s1, s2, s3, shadow, cfg[2], step)
        assert torch.count_nonzero(gg) == 0  # zeroed for the next step
    torch.cuda.synchronize()
    assert int(step.item()) == len(grads)
    close(p, ref.detach(), rtol=1e-5, atol=1e-5)
    close(shadow, ref.detach())
    if name == "rmsprop_plain":
        assert torch.count_nonzero(s2) == 0 and torch.count_nonzero(s3) == 0  # never touched


def test_dropout_mask_reuse():
    x = bf(torch.ones(1 << 20, device=dev))
    rng = torch.tensor([1234, 0], device=dev, dtype=torch.int64)
    y = K.dropout(x, 0.3, rng, salt=7)
    keep = (y.float() != 0).float().mean().item()
    assert abs(keep - 0.7) < 0.01
    assert torch.allclose(y.float()[y.float() != 0], torch.full_like(y.float()[y.float() != 0], 1 / 0.7), rtol=1e-2)
    dy = K.dropout(x, 0.3, rng, salt=7)
    assert torch.equal(dy, y)  # backward regenerates the same mask
    K.rng_advance(rng)
    y2 = K.dropout(x, 0.3, rng, salt=7)
    assert not torch.equal(y2, y)


@pytest.mark.parametrize("M,C", [(4096, 96), (8192, 64), (3136, 2048), (1000, 16), (50001, 256), (131072, 16),
                                 (32768, 32)])
def test_batchnorm(M, C):
    """Vectorized (C/8 | 256) and scalar (C = 96) BN paths; run twice so the zero-at-rest
    replica accumulators must have been re-zeroed by the first call's finalize kernels."""
    torch.manual_seed(7)
    x = bf(torch.randn(M, C, device=dev) * 2 + 1)
    res = bf(torch.randn(M, C, device=dev))
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.randn(C, device=dev)
    mean = torch.empty(C, device=dev)
    rstd = torch.empty(C, device=dev)
    rm = torch.zeros(C, device=dev)
    rv = torch.ones(C, device=dev)
    y = K.bn_fwd_train(x, gamma, beta, mean, rstd, rm, rv, 0.1, 1e-5, residual=res, act="relu")
    rm.zero_()
    rv.fill_(1.0)
    y = K.bn_fwd_train(x, gamma, beta, mean, rstd, rm, rv, 0.1, 1e-5, residual=res, act="relu")
    xr = x.float().requires_grad_(True)
    gr = gamma.clone().requires_grad_(True)
    br = beta.clone().requires_grad_(True)
    rr = res.float().requires_grad_(True)
    rm2, rv2 = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    yr = (F.batch_norm(xr, rm2, rv2, gr, br, True, 0.1, 1e-5) + rr).relu()
    close(y, yr)
    close(rm, rm2, rtol=1e-3, atol=1e-4)
    close(rv, rv2, rtol=1e-3, atol=1e-4)
    dy = bf(torch.randn(M, C, device=dev))
    gx, gg, gb, grr = torch.autograd.grad(yr, (xr, gr, br, rr), dy.float())
    dg = torch.zeros(C, device=dev)
    db = torch.zeros(C, device=dev)
    ws = torch.empty(2 * C, device=dev)
    dres = torch.empty_like(x)
    dx = K.bn_bwd(dy, x, y, gamma, mean, rstd, dg, db, ws, act="relu", dresidual=dres)
    dg.zero_()
    db.zero_()
    dx = K.bn_bwd(dy, x, y, gamma, mean, rstd, dg, db, ws, act="relu", dresidual=dres)
    close(dx, gx, rtol=3e-2, atol=3e-2)
    close(dg, gg, rtol=3e-2, atol=3e-2)
    close(db, gb, rtol=3e-2, atol=3e-2)
    close(dres, grr)
    if C % 8 == 0:  # the one-launch backward's grid barrier never timed out
        torch.cuda.synchronize()
        assert K.bn_coop_timeouts(torch.device(dev), C) == 0


@pytest.mark.parametrize("M,C", [(4096, 64), (2048, 256), (512, 2048)])
def test_batchnorm_bwd_zmask(M, C):
    """ReLU BN without residual: the backward's act' mask recomputed from x (zbeta, norm.hip bn_shift)
    gives the y-read path's result, and matches PyTorch."""
    torch.manual_seed(9)
    x = bf(torch.randn(M, C, device=dev) * 2 + 0.3)
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.randn(C, device=dev)
    mean, rstd = torch.empty(C, device=dev), torch.empty(C, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    y = K.bn_fwd_train(x, gamma, beta, mean, rstd, rm, rv, 0.1, 1e-5, act="relu")
    dy = bf(torch.randn(M, C, device=dev))
    outs = []
    for zb in (None, beta):
        dg, db, ws = torch.zeros(C, device=dev), torch.zeros(C, device=dev), torch.empty(2 * C, device=dev)
        dx = K.bn_bwd(dy, x, y, gamma, mean, rstd, dg, db, ws, act="relu", zbeta=zb)
        outs.append((dx, dg, db))
    (dx0, dg0, db0), (dx1, dg1, db1) = outs
    close(dx1, dx0, rtol=1e-2, atol=1e-2)  # the same mask; the column sums differ by float-atomic order only
    torch.testing.assert_close(dg1, dg0, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(db1, db0, rtol=1e-5, atol=1e-4)
    xr = x.float().requires_grad_(True)
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    yr = F.batch_norm(xr, None, None, gr, br, True, 0.1, 1e-5).relu()
    gx, gg, gb = torch.autograd.grad(yr, (xr, gr, br), dy.float())
    close(dx1, gx, rtol=3e-2, atol=3e-2)
    close(dg1, gg, rtol=3e-2, atol=3e-2)
    close(db1, gb, rtol=3e-2, atol=3e-2)


def test_embedding_bag():
    torch.manual_seed(8)
    V, D = 1000, 24
    table = torch.randn(V, D, device=dev)
    idx = torch.randint(0, V, (300,), device=dev)
    offs = torch.tensor(sorted(torch.randint(0, 300, (63,)).tolist()), device=dev)
    offs[0] = 0
    for mode in (0, 1):
        out = torch.zeros(63, 40, device=dev)
        K.embedding_bag_fwd(table, idx, offs, mode, out[:, 8:32], ldo=40)
        ref = F.embedding_bag(idx, table, offs, mode="sum" if mode == 0 else "mean")
        close(out[:, 8:32], ref, rtol=1e-5, atol=1e-5)
        dout = torch.randn(63, 40, device=dev)
        dt = torch.zeros_like(table)
        K.embedding_bag_bwd(dout[:, 8:32], idx, offs, mode, dt, 63, ldo=40)
        tr = table.clone().requires_grad_(True)
        (g,) = torch.autograd.grad(F.embedding_bag(idx, tr, offs, mode="sum" if mode == 0 else "mean"), (tr,),
                                   dout[:, 8:32])
        close(dt, g, rtol=1e-4, atol=1e-5)


def test_column_stats():
    torch.manual_seed(9)
    x = torch.randn(10007, 37, device=dev) * 3 + 2
    x[5, 3] = float("nan")
    st = K.column_stats(x)
    m = ~torch.isnan(x)
    xz = torch.where(m, x, torch.zeros_like(x))
    close(st[:, 0], m.sum(0).float(), rtol=0, atol=1e-3)
    close(st[:, 1], xz.sum(0), rtol=1e-4, atol=1e-2)
    xi = torch.where(m, x, torch.full_like(x, float("inf")))
    xa = torch.where(m, x, torch.full_like(x, float("-inf")))
    assert torch.equal(st[:, 3], xi.min(0).values) and torch.equal(st[:, 4], xa.max(0).values)
    h = K.column_hist(x, st[:, 3].contiguous(), st[:, 4].contiguous(), 20)
    assert h.sum(1).tolist() == m.sum(0).tolist()
    mean = (st[:, 1] / st[:, 0]).contiguous()
    g = K.gram(x, mean)
    xc = (xz - mean) * m
    close(g, xc.t() @ xc, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("B,H,W,C,k", [(32, 26, 26, 64, 2), (16, 27, 27, 32, 2), (8, 22, 22, 64, 4)])
def test_maxpool_fused_dropout_act(B, H, W, C, k):
    """pool -> dropout fused forward; backward re-applies the mask, relu' of the pool input and the bias-grad sum."""
    torch.manual_seed(10)
    x = bf(torch.randn(B, H, W, C, device=dev)).relu()
    rng = torch.tensor([99, 3], device=dev, dtype=torch.int64)
    p = 0.3
    y, am = K.maxpool2d_fwd(x, (k, k), (k, k), (0, 0), drop_p=p, rng=rng, salt=5)
    y0, _ = K.maxpool2d_fwd(x, (k, k), (k, k), (0, 0))
    mask = (y.float() != 0) | (y0.float() == 0)
    keep = (y.float() != 0).float().sum() / (y0.float() != 0).float().sum()
    assert abs(keep.item() - (1 - p)) < 0.05
    torch.testing.assert_close(y.float()[y.float() != 0], (y0.float() / (1 - p))[y.float() != 0], rtol=1e-2, atol=1e-2)
    dy = bf(torch.randn_like(y.float()))
    cs = torch.zeros(C, device=dev)
    dx = K.maxpool2d_bwd(dy, am, x.shape, (k, k), (k, k), (0, 0), x=x, act="relu", colsum=cs, drop_p=p, rng=rng,
                         salt=5)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.max_pool2d(xr, k, k)
    dmask = ((y.float() != 0) & (y0.float() != 0)) | ((y0.float() == 0) & (y.float() == 0))
    drop = torch.where(y.float() != 0, torch.full_like(dy.float(), 1 / (1 - p)), torch.zeros_like(dy.float()))
    # for windows whose max is 0 the mask is ambiguous from outputs; relu' kills them anyway
    (gx,) = torch.autograd.grad(yr, (xr,), (dy.float() * drop).permute(0, 3, 1, 2))
    ref = gx.permute(0, 2, 3, 1) * (x.float() > 0)
    close(dx, ref)
    close(cs, ref.sum((0, 1, 2)), rtol=3e-2, atol=3e-2)
    del mask, dmask
