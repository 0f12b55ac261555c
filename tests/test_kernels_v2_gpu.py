"""Numerics of the second-generation kernels vs fp32 PyTorch references: small-K conv weight
gradient (register-accumulated, shuffle/LDS reduced) with the fused act' mask, and the uint8
input layer with its normalisation fused into the direct forward and the wgrad kernels."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd.ops import kernels as K  # noqa: E402

dev = torch.device("cuda", 0)
bf = torch.bfloat16


def _ref_wgrad(dy, x, k, act_y=None):
    # dy [B,OH,OW,CO] (bf16 values), x [B,H,W,C] float; returns dW [CO,KH,KW,C], db [CO]
    d = dy.float()
    if act_y is not None:
        d = d * (act_y.float() > 0).float()
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(False)
    CO = d.shape[-1]
    w = torch.zeros(CO, x.shape[-1], k, k, device=dev, requires_grad=True)
    out = F.conv2d(xr, w)
    out.backward(d.permute(0, 3, 1, 2))
    return w.grad.permute(0, 2, 3, 1).reshape(CO, -1), d.sum((0, 1, 2))


@pytest.mark.parametrize("k,C,CO,B,H", [(2, 1, 32, 32, 28), (3, 1, 32, 7, 28), (4, 1, 32, 5, 28), (2, 4, 16, 3, 20),
                                        (3, 1, 64, 2, 12)])
@pytest.mark.parametrize("masked", [False, True])
def test_smallk_wgrad(k, C, CO, B, H, masked):
    torch.manual_seed(0)
    x = torch.randn(B, H, H, C, device=dev).to(bf)
    OH = H - k + 1
    dy = torch.randn(B, OH, OH, CO, device=dev).to(bf)
    y = torch.relu(torch.randn(B, OH, OH, CO, device=dev)).to(bf) if masked else None
    g = K.conv_geom(x.shape, (CO, k, k, C), (1, 1), (0, 0), (1, 1))
    dw = torch.zeros(CO, k * k * C, device=dev)
    db = torch.zeros(CO, device=dev)
    K.conv2d_wgrad(dy, x, g, dw, dbias=db, y=y, act="relu" if masked else 0)
    rw, rb = _ref_wgrad(dy, x, k, y)
    torch.testing.assert_close(dw, rw, atol=2e-2 * rw.abs().max().item(), rtol=1e-2)
    torch.testing.assert_close(db, rb, atol=2e-2 * rb.abs().max().item() + 1e-3, rtol=1e-2)


@pytest.mark.parametrize("k,CO,B,stride,pad", [(4, 32, 32, 1, 0), (5, 16, 8, 1, 2), (3, 64, 4, 2, 1), (2, 8, 9, 1, 0)])
def test_c1_wgrad_pixel_range_kernel(k, CO, B, stride, pad, monkeypatch):
    """conv_wgrad_c1_k (one-channel input layers: the E1 model's 4x4 conv at batch 32 first) against the fp32
    reference for three different inputs in a row (the in-launch combine hands rows between workgroups and
    XCDs through write-through stores: stale rows would show as a wrong sum), and bit-identical when an input
    is repeated (two-level ordered combine; a one-atomic-per-workgroup combine measured 36.4 vs 32.0 us)."""
    torch.manual_seed(7)
    H = 28
    sc, sh = 1 / 255.0, -0.5
    g = K.conv_geom((B, H, H, 1), (CO, k, k, 1), (stride, stride), (pad, pad), (1, 1))
    OH, OW = g[4], g[5]
    ins = [(torch.randint(0, 256, (B, H, H, 1), dtype=torch.uint8, device=dev),
            torch.randn(B, OH, OW, CO, device=dev).to(bf), torch.relu(torch.randn(B, OH, OW, CO, device=dev)).to(bf))
           for _ in range(3)]
    outs = []
    for xu, dy, y in ins + ins[:1]:
        dw = torch.zeros(CO, k * k, device=dev)
        db = torch.zeros(CO, device=dev)
        K.conv2d_wgrad(dy, xu, g, dw, dbias=db, y=y, act="relu", in_affine=(sc, sh))
        outs.append((dw, db))
    assert torch.equal(outs[0][0], outs[3][0]) and torch.equal(outs[0][1], outs[3][1])
    for (xu, dy, y), (dw, db) in zip(ins, outs):
        d = dy.float() * (y.float() > 0).float()
        wr = torch.zeros(CO, 1, k, k, device=dev, requires_grad=True)
        xf = (xu.float() * sc + sh).permute(0, 3, 1, 2)
        F.conv2d(xf, wr, stride=stride, padding=pad).backward(d.permute(0, 3, 1, 2))
        rw = wr.grad.permute(0, 2, 3, 1).reshape(CO, -1)
        torch.testing.assert_close(dw, rw, atol=1e-3 * rw.abs().max().item(), rtol=1e-3)
        torch.testing.assert_close(db, d.sum((0, 1, 2)), atol=1e-3 * d.sum((0, 1, 2)).abs().max().item(), rtol=1e-3)


@pytest.mark.parametrize("k", [2, 3, 4])
def test_u8_fused_input_layer(k):
    torch.manual_seed(1)
    B, H, CO = 16, 28, 32
    xu = torch.randint(0, 256, (B, H, H, 1), dtype=torch.uint8, device=dev)
    sc, sh = 1 / 255.0, -0.5
    xf = xu.float() * sc + sh
    w = (torch.randn(CO, k, k, 1, device=dev) * 0.3).to(bf)
    b = torch.randn(CO, device=dev) * 0.1
    g = K.conv_geom(xu.shape, w.shape, (1, 1), (0, 0), (1, 1))
    assert K.conv_u8_fusable(g)
    y = K.conv2d_fwd(xu, w, g, bias=b, act="relu", in_affine=(sc, sh))
    ref = torch.relu(F.conv2d(xf.permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b)).permute(0, 2, 3, 1)
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=2e-2)
    dy = torch.randn_like(y)
    dw = torch.zeros(CO, k * k, device=dev)
    K.conv2d_wgrad(dy, xu, g, dw, y=y, act="relu", in_affine=(sc, sh))
    rw, _ = _ref_wgrad(dy, xf, k, y)
    torch.testing.assert_close(dw, rw, atol=2e-2 * rw.abs().max().item(), rtol=1e-2)


def test_mnist_models_use_fused_input_path():
    from hops_examples_amd.models.mnist import MirroredMnistCNN, TorchMnistNet
    from hops_examples_amd.ops import functional as HF
    from hops_examples_amd.runtime.arena import ParamArena

    for cls in (MirroredMnistCNN, TorchMnistNet):  # fused (K=4) and unfused (K=25) input layers
        torch.manual_seed(0)
        cpu = cls()
        gpu = cls().to(dev)
        gpu.load_state_dict(cpu.state_dict())
        ParamArena.from_module(gpu)
        x = torch.randint(0, 256, (8, 28, 28, 1), dtype=torch.uint8)
        y = torch.randint(0, 10, (8,))
        lc = HF.loss(cpu.eval()(x), y)
        lg = HF.loss(gpu.eval()(x.to(dev)), y.to(dev))
        assert abs(lc.item() - lg.item()) < 0.03 * max(1.0, lc.item()), (cls.__name__, lc.item(), lg.item())


def _torch_conv(x, w, b, pad):
    return F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, padding=pad).permute(0, 2, 3, 1)


@pytest.mark.parametrize("k,C,CO,H,pad", [(2, 32, 64, 27, 0), (3, 32, 64, 28, 1), (4, 32, 64, 25, 0), (2, 16, 32, 9, 0),
                                          (3, 64, 128, 10, 1), (1, 64, 16, 7, 0), (3, 16, 16, 12, 1), (3, 16, 32, 8, 1)])
def test_conv_mfma_fwd(k, C, CO, H, pad):
    torch.manual_seed(2)
    B = 3
    x = torch.randn(B, H, H, C, device=dev).to(bf)
    w = (torch.randn(CO, k, k, C, device=dev) * 0.1).to(bf)
    b = torch.randn(CO, device=dev) * 0.1
    g = K.conv_geom(x.shape, w.shape, (1, 1), (pad, pad), (1, 1))
    y = K.conv2d_fwd(x, w, g, bias=b, act="relu")
    ref = torch.relu(_torch_conv(x, w, b, pad))
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("k,C,CO,H,pad,B,masked", [(2, 32, 64, 27, 0, 2, True), (3, 32, 64, 14, 1, 2, True),
                                                   (4, 32, 64, 13, 0, 2, True), (2, 16, 32, 9, 0, 2, True),
                                                   (3, 16, 16, 12, 1, 2, True),
                                                   # K = 16 x 64 = 1024 (32 K-steps): the E1 model's conv2
                                                   (4, 32, 64, 25, 0, 32, False), (4, 32, 64, 25, 0, 3, True),
                                                   (4, 16, 64, 11, 1, 4, True), (5, 32, 40, 9, 2, 2, False)])
def test_conv_mfma_dgrad_masks_colsum(k, C, CO, H, pad, B, masked):
    torch.manual_seed(3)
    xprev = torch.relu(torch.randn(B, H, H, C, device=dev)).to(bf)  # previous layer's activation output
    w = (torch.randn(CO, k, k, C, device=dev) * 0.1).to(bf)
    g = K.conv_geom(xprev.shape, w.shape, (1, 1), (pad, pad), (1, 1))
    OH = g[4]
    y = torch.relu(torch.randn(B, OH, OH, CO, device=dev)).to(bf)
    dy = torch.randn(B, OH, OH, CO, device=dev).to(bf)
    if not masked:  # pre-masked dY (the fused pool backward applied ReLU'): no y operand
        dy = (dy.float() * (y.float() > 0)).to(bf)
    cs = torch.zeros(C, device=dev)
    dx = K.conv2d_dgrad(dy, w, g, yprev=xprev, act_prev="relu", colsum=cs, y=y if masked else None,
                        act="relu" if masked else 0)
    xr = xprev.float().permute(0, 3, 1, 2).clone().requires_grad_(True)
    out = F.conv2d(xr, w.float().permute(0, 3, 1, 2), padding=pad)
    out.backward((dy.float() * (y.float() > 0)).permute(0, 3, 1, 2))
    ref = xr.grad.permute(0, 2, 3, 1) * (xprev.float() > 0)
    torch.testing.assert_close(dx.float(), ref, atol=3e-2 * ref.abs().max().item(), rtol=2e-2)
    torch.testing.assert_close(cs, ref.sum((0, 1, 2)), atol=3e-2 * ref.abs().sum((0, 1, 2)).max().item() + 1e-2,
                               rtol=3e-2)


@pytest.mark.parametrize("k0,pad0,C,CO,k,u8", [(2, 0, 32, 64, 2, True), (2, 0, 32, 64, 2, False),
                                               (3, 1, 16, 32, 2, True), (3, 1, 64, 32, 2, False),
                                               (2, 0, 32, 16, 3, True)])
def test_dgrad_fused_input_layer_wgrad(k0, pad0, C, CO, k, u8):
    """conv(g) dgrad carrying the input layer conv(g0) weight/bias gradient (no dX written):
    compared with an fp32 autograd reference of the two-layer chain."""
    torch.manual_seed(4)
    B, H = 3, 20
    sc, sh = (1 / 255.0, -0.5) if u8 else (None, None)
    if u8:
        x0 = torch.randint(0, 256, (B, H, H, 1), dtype=torch.uint8, device=dev)
        x0f = x0.float() * sc + sh
    else:
        x0 = torch.randn(B, H, H, 1, device=dev).to(bf)
        x0f = x0.float()
    w0 = (torch.randn(C, k0, k0, 1, device=dev) * 0.5).to(bf)
    b0 = torch.randn(C, device=dev) * 0.1
    g0 = K.conv_geom(x0.shape, w0.shape, (1, 1), (pad0, pad0), (1, 1))
    y0 = K.conv2d_fwd(x0, w0, g0, bias=b0, act="relu", in_affine=(sc, sh) if u8 else None)
    w = (torch.randn(CO, k, k, C, device=dev) * 0.1).to(bf)
    g = K.conv_geom(y0.shape, w.shape, (1, 1), (0, 0), (1, 1))
    assert K.conv_dgrad_fused_wgrad_ok(g, g0)
    OH = g[4]
    y = torch.relu(torch.randn(B, OH, OH, CO, device=dev)).to(bf)
    dy = torch.randn(B, OH, OH, CO, device=dev).to(bf)
    dw0 = torch.zeros(C, k0 * k0, device=dev)
    db0 = torch.zeros(C, device=dev)
    K.conv2d_dgrad_fused_wgrad(dy, w, g, y0, "relu", y, "relu", x0, g0, dw0, db0,
                               in_affine=(sc, sh) if u8 else None)
    # reference: dX1 = conv^T(dy * relu'(y)) masked by relu'(y0), then the input layer's wgrad
    xr = y0.float().permute(0, 3, 1, 2).clone().requires_grad_(True)
    F.conv2d(xr, w.float().permute(0, 3, 1, 2)).backward((dy.float() * (y.float() > 0)).permute(0, 3, 1, 2))
    d1 = (xr.grad.permute(0, 2, 3, 1) * (y0.float() > 0)).to(bf).float()  # the kernel masks bf16 dX
    wr = torch.zeros(C, 1, k0, k0, device=dev, requires_grad=True)
    F.conv2d(x0f.permute(0, 3, 1, 2), wr, padding=pad0).backward(d1.permute(0, 3, 1, 2))
    rw = wr.grad.permute(0, 2, 3, 1).reshape(C, -1)
    torch.testing.assert_close(dw0, rw, atol=2e-2 * rw.abs().max().item(), rtol=2e-2)
    torch.testing.assert_close(db0, d1.sum((0, 1, 2)), atol=2e-2 * d1.abs().sum((0, 1, 2)).max().item() + 1e-3,
                               rtol=2e-2)


def test_mirrored_cnn_fused_input_wgrad_matches_unfused(monkeypatch):
    """MirroredMnistCNN's conv1 weight gradient comes out of conv2's dgrad launch; the gradients
    must equal the unfused path (separate dX + small-K wgrad) up to bf16 rounding."""
    from hops_examples_amd.models.mnist import MirroredMnistCNN
    from hops_examples_amd.ops import functional as HF
    from hops_examples_amd.runtime.arena import ParamArena

    grads = []
    for disable in ("", "fused_wgrad0"):
        monkeypatch.setenv("HOPSX_DISABLE", disable)
        HF.seed_device_rng(7, dev)  # same dropout mask in both runs
        torch.manual_seed(0)
        m = MirroredMnistCNN().to(dev)
        m.pool.salt = 7919  # per-instance dropout salt: pin it
        ParamArena.from_module(m, dev)
        x = torch.randint(0, 256, (16, 28, 28, 1), dtype=torch.uint8, device=dev)
        t = torch.randint(0, 10, (16,), device=dev)
        out = m(x)
        _, _, _, dl = HF.loss_and_grad(out, t, "sparse_ce")
        out.backward(dl)
        torch.cuda.synchronize()
        assert m.conv1.weight._hx_grad.abs().sum().item() > 0
        grads.append(m._hx_arena.grad.float().clone())
    a, b = grads
    torch.testing.assert_close(a, b, atol=2e-2 * b.abs().max().item(), rtol=2e-2)


@pytest.mark.parametrize("k,C,CO,H,pad,stride", [(2, 32, 64, 27, 0, 1), (3, 16, 16, 16, 1, 1), (1, 64, 16, 7, 0, 1),
                                                 (3, 8, 64, 11, 1, 1), (3, 16, 32, 16, 1, 2), (2, 32, 32, 5, 0, 1)])
@pytest.mark.parametrize("masked", [False, True])
def test_conv_wgrad_mfma(k, C, CO, H, pad, stride, masked):
    """Direct MFMA weight gradient (wave-private LDS images read back with ds_read_b64_tr_b16)."""
    torch.manual_seed(5)
    B = 3
    x = torch.randn(B, H, H, C, device=dev).to(bf)
    g = K.conv_geom(x.shape, (CO, k, k, C), (stride, stride), (pad, pad), (1, 1))
    OH, OW = g[4], g[5]
    dy = torch.randn(B, OH, OW, CO, device=dev).to(bf)
    y = torch.relu(torch.randn(B, OH, OW, CO, device=dev)).to(bf) if masked else None
    dw = torch.zeros(CO, k * k * C, device=dev)
    db = torch.zeros(CO, device=dev)
    K.conv2d_wgrad(dy, x, g, dw, dbias=db, y=y, act="relu" if masked else 0)
    d = dy.float() * ((y.float() > 0).float() if masked else 1.0)
    wr = torch.zeros(CO, C, k, k, device=dev, requires_grad=True)
    F.conv2d(x.float().permute(0, 3, 1, 2), wr, stride=stride, padding=pad).backward(d.permute(0, 3, 1, 2))
    rw = wr.grad.permute(0, 2, 3, 1).reshape(CO, -1)
    torch.testing.assert_close(dw, rw, atol=2e-2 * rw.abs().max().item(), rtol=1e-2)
    rb = d.sum((0, 1, 2))
    torch.testing.assert_close(db, rb, atol=2e-2 * rb.abs().max().item() + 1e-3, rtol=1e-2)


def test_pool_premask_matches_conv_mask(monkeypatch):
    """conv(ReLU) -> max-pool: the ReLU' mask moved into the pool backward gives the same
    gradients as the conv applying it itself."""
    from hops_examples_amd.models.mnist import MirroredMnistCNN
    from hops_examples_amd.ops import functional as HF
    from hops_examples_amd.runtime.arena import ParamArena

    grads = []
    for disable in ("", "premask"):
        monkeypatch.setenv("HOPSX_DISABLE", disable)
        HF.seed_device_rng(11, dev)
        torch.manual_seed(0)
        m = MirroredMnistCNN().to(dev)
        m.pool.salt = 7919
        ParamArena.from_module(m, dev)
        x = torch.randint(0, 256, (16, 28, 28, 1), dtype=torch.uint8, device=dev)
        t = torch.randint(0, 10, (16,), device=dev)
        out = m(x)
        _, _, _, dl = HF.loss_and_grad(out, t, "sparse_ce")
        out.backward(dl)
        torch.cuda.synchronize()
        grads.append(m._hx_arena.grad.float().clone())
    assert not HF._PREMASKED
    torch.testing.assert_close(grads[0], grads[1], atol=2e-2 * grads[1].abs().max().item(), rtol=2e-2)


@pytest.mark.parametrize("dtype,n", [(torch.float32, 1), (torch.float32, 100003), (bf, 4097), (bf, 1 << 20)])
def test_nonfinite_counts(dtype, n):
    """hopsx_nonfinite (health pill) vs torch.isnan / isinf."""
    torch.manual_seed(6)
    x = torch.randn(n, device=dev).to(dtype)
    idx = torch.randperm(n, device=dev)
    x[idx[: n // 7]] = float("nan")
    x[idx[n // 7: n // 7 + n // 11]] = float("inf")
    x[idx[n // 7 + n // 11: n // 7 + n // 11 + n // 13]] = float("-inf")
    c = K.nonfinite_counts(x).cpu()
    assert int(c[0]) == int(torch.isnan(x.float()).sum()) and int(c[1]) == int(torch.isinf(x.float()).sum())


def test_step_profiler_captures_hip_kernels(tmp_path):
    """torch.profiler (roctracer) sees the hopsx kernels by name inside the step window."""
    from hops_examples_amd import profiler

    x = torch.randn(4096, device=dev)
    with profiler.profile("1,2", logdir=str(tmp_path), run_name="g") as p:
        for _ in range(3):
            K.nonfinite_counts(x)
            p.step()
    names = [r["name"] for r in profiler.trace_kernel_summary(p.trace_path)]
    assert any("nonfinite_k" in n for n in names), names[:10]


@pytest.mark.parametrize("B,H,C,k,s,p", [(4, 112, 64, 3, 2, 1), (3, 15, 16, 3, 2, 1), (2, 9, 32, 2, 1, 0),
                                         (2, 14, 8, 3, 3, 1)])
@pytest.mark.parametrize("act", [0, 1])
def test_maxpool_vectorized_general(B, H, C, k, s, p, act):
    """Overlapping / padded windows on the 16-B general kernels (ResNet stem 3x3/2 pad 1), bwd
    without colsum, with the fused ReLU' of the pool input."""
    torch.manual_seed(8)
    x = torch.relu(torch.randn(B, H, H, C, device=dev)).to(bf) if act else torch.randn(B, H, H, C, device=dev).to(bf)
    y, am = K.maxpool2d_fwd(x, (k, k), (s, s), (p, p))
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.max_pool2d(xr, k, s, p)
    torch.testing.assert_close(y.float(), yr.permute(0, 2, 3, 1), rtol=0, atol=1e-6)
    dy = torch.randn_like(y.float()).to(bf)
    (gx,) = torch.autograd.grad(yr, (xr,), dy.float().permute(0, 3, 1, 2))
    gx = gx.permute(0, 2, 3, 1)
    if act:
        gx = gx * (x.float() > 0)
    dx = K.maxpool2d_bwd(dy, am, x.shape, (k, k), (s, s), (p, p), x=x if act else None, act="relu" if act else 0)
    torch.testing.assert_close(dx.float(), gx, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("B,HW,C", [(64, 49, 2048), (3, 64, 16), (5, 1, 64)])
def test_global_avg_pool_vectorized(B, HW, C):
    torch.manual_seed(9)
    x = torch.randn(B, HW, 1, C, device=dev).to(bf)
    y = K.gap_fwd(x.view(B, HW, 1, C))
    torch.testing.assert_close(y.float(), x.float().mean((1, 2)), rtol=1e-2, atol=1e-2)
    dy = torch.randn(B, C, device=dev).to(bf)
    dx = K.gap_bwd(dy, (B, HW, 1, C))
    torch.testing.assert_close(dx.float(), (dy.float() / HW)[:, None, None, :].expand(B, HW, 1, C), rtol=1e-2,
                               atol=1e-3)


def test_plain_1x1_conv_library_gemm_matches_kernel(monkeypatch):
    """Epilogue-free 1x1 convs run as hipBLASLt GEMMs (bf16 in, fp32 weight-grad out); gradients
    must match the MFMA implicit-GEMM path."""
    from hops_examples_amd.ops import functional as HF

    torch.manual_seed(10)
    x0 = torch.randn(4, 32, 32, 64, device=dev).to(bf)
    w0 = torch.randn(128, 1, 1, 64, device=dev) * 0.1
    dy = torch.randn(4, 32, 32, 128, device=dev).to(bf)
    outs = []
    for disable in ("", "blaslt_1x1"):
        monkeypatch.setenv("HOPSX_DISABLE", disable)
        x = x0.clone().requires_grad_(True)
        w = w0.clone().requires_grad_(True)
        y = HF.conv2d(x, w)
        y.backward(dy)
        outs.append((y.float(), x.grad.float(), w.grad.float()))
    for a, b in zip(*outs):
        torch.testing.assert_close(a, b, atol=2e-2 * b.abs().max().item(), rtol=2e-2)


# B = 200: 7 row blocks (loss totals summed from per-block slots by the last to arrive); B = 2100: 66 row
# blocks (more than the slots: zeroed totals + atomics)
@pytest.mark.parametrize("kind,C,B", [("sparse_ce", 10, 32), ("sparse_ce", 10, 200), ("ce", 10, 17),
                                      ("bce_logits", 1, 40), ("mse", 3, 9), ("sparse_ce", 10, 2100)])
def test_fused_classifier_head(monkeypatch, kind, C, B):
    """loss_and_grad_root on a linear logits layer: one head_ce launch (loss, dW, db, dh) must give
    the same loss and gradients as the loss kernel + the layer's backward GEMMs."""
    from hops_examples_amd.ops import functional as HF
    from hops_examples_amd.runtime.arena import ParamArena

    torch.manual_seed(11)
    h0 = torch.randn(B, 128, device=dev).to(bf)
    if kind == "sparse_ce":
        t = torch.randint(0, C, (B,), device=dev)
    elif kind == "ce":
        t = torch.nn.functional.one_hot(torch.randint(0, C, (B,), device=dev), C).float()
    else:
        t = torch.rand(B, C, device=dev).round() if kind == "bce_logits" else torch.randn(B, C, device=dev)
    res = []
    for disable in ("", "head_ce"):
        monkeypatch.setenv("HOPSX_DISABLE", disable)
        lin = torch.nn.Linear(128, C).to(dev)
        with torch.no_grad():
            torch.manual_seed(12)
            lin.weight.copy_(torch.randn(C, 128, device=dev) * 0.1)
            lin.bias.copy_(torch.randn(C, device=dev) * 0.1)
        ParamArena.from_module(lin, dev)
        h = h0.clone().requires_grad_(True)
        out = HF.linear(h, lin.weight, lin.bias, out_f32=True)
        loss, correct, count, root, grad = HF.loss_and_grad_root(out, t, kind)
        assert (root is h) == (disable == "")
        root.backward(grad)
        torch.cuda.synchronize()
        res.append((loss.clone(), correct.clone(), lin._hx_arena.grad.clone(), h.grad.float().clone()))
    (l0, c0, g0, d0), (l1, c1, g1, d1) = res
    torch.testing.assert_close(l0, l1, rtol=1e-4, atol=1e-5)
    assert int(c0) == int(c1)
    monkeypatch.setenv("HOPSX_DISABLE", "")
    for _ in range(2):  # more launches: the row-block slots' arrival counter is back at zero after each
        out2 = HF.linear(h0.clone().requires_grad_(True), lin.weight, lin.bias, out_f32=True)
        loss2, correct2 = HF.loss_and_grad_root(out2, t, kind)[:2]
        torch.cuda.synchronize()
        torch.testing.assert_close(loss2, l1, rtol=1e-4, atol=1e-5)
        assert int(correct2) == int(c1)
    torch.testing.assert_close(g0, g1, rtol=2e-2, atol=2e-2 * g1.abs().max().item())
    torch.testing.assert_close(d0, d1, rtol=2e-2, atol=2e-2 * d1.abs().max().item())


@pytest.mark.parametrize("model", ["mirrored", "cifar"])
def test_paired_conv_backward_matches_separate_launches(monkeypatch, model):
    """conv_bwd_pair_k (dgrad + wgrad workgroups in one launch) vs the two separate launches."""
    from hops_examples_amd.models.mnist import MirroredMnistCNN
    from hops_examples_amd.models.resnet import cifar_resnet
    from hops_examples_amd.ops import functional as HF
    from hops_examples_amd.runtime.arena import ParamArena

    grads = []
    for disable in ("", "bwd_pair", ""):
        monkeypatch.setenv("HOPSX_DISABLE", disable)
        HF.seed_device_rng(3, dev)
        torch.manual_seed(0)
        if model == "mirrored":
            m = MirroredMnistCNN().to(dev)
            m.pool.salt = 7919
            x = torch.randint(0, 256, (32, 28, 28, 1), dtype=torch.uint8, device=dev)
        else:
            m = cifar_resnet(20).to(dev)
            x = torch.randint(0, 256, (16, 32, 32, 3), dtype=torch.uint8, device=dev)
        ParamArena.from_module(m, dev)
        t = torch.randint(0, 10, (x.shape[0],), device=dev)
        out = m(x)
        _, _, _, root, g = HF.loss_and_grad_root(out, t, "sparse_ce")
        root.backward(g)
        torch.cuda.synchronize()
        grads.append(m._hx_arena.grad.float().clone())
    if model == "mirrored":
        torch.testing.assert_close(grads[0], grads[1], atol=3e-2 * grads[1].abs().max().item(), rtol=3e-2)
    else:
        # BatchNorm statistics are float-atomic sums (run-to-run last-bit noise that 20 layers of BN
        # backward amplify): the pair must agree with the separate launches as well as a rerun does
        cos = lambda a, b: float(torch.nn.functional.cosine_similarity(a, b, dim=0))  # noqa: E731
        noise, diff = cos(grads[0], grads[2]), cos(grads[0], grads[1])
        # (with deterministic BN sums a rerun is near bit-exact, so the relative bound is capped:
        # the pair and the separate launches still sum in a different order)
        assert diff > 0.97 and diff > min(noise, 0.99) - 0.02, (diff, noise)
        # the tight criterion is per layer (whole steps differ by the network's sensitivity to any sum
        # order): both forms against fp64 at their own operating point, every tensor > 0.999
        from hops_examples_amd.runtime import layercheck as LC

        for dis in ("", "bwd_pair"):
            r = LC.resnet20_check(16, dis)
            assert r["min_grad_cos"] > 0.999, (dis, r["min_grad_cos"])


@pytest.mark.parametrize("model", ["mirrored", "torch"])
def test_pool_backward_fused_into_linear_dgrad(monkeypatch, model):
    """Max-pool (+dropout, +ReLU' premask) -> flatten -> Linear: the pool backward done by the
    Linear's dgrad epilogue (EpiPoolScatterBF16) equals the separate pool-backward launch."""
    from hops_examples_amd.models import mnist
    from hops_examples_amd.ops import functional as HF
    from hops_examples_amd.runtime.arena import ParamArena

    grads = []
    for disable in ("", "pool_scatter"):
        monkeypatch.setenv("HOPSX_DISABLE", disable)
        calls = []
        real = K.maxpool2d_bwd
        monkeypatch.setattr(K, "maxpool2d_bwd", lambda *a, **kw: calls.append(1) or real(*a, **kw))
        HF.seed_device_rng(5, dev)
        torch.manual_seed(0)
        m = (mnist.MirroredMnistCNN() if model == "mirrored" else mnist.TorchMnistNet()).to(dev)
        for mod in m.modules():
            if hasattr(mod, "salt"):
                mod.salt = 7919
        ParamArena.from_module(m, dev)
        x = torch.randint(0, 256, (32, 28, 28, 1), dtype=torch.uint8, device=dev)
        t = torch.randint(0, 10, (32,), device=dev)
        out = m(x)
        _, _, _, root, g = HF.loss_and_grad_root(out, t, "sparse_ce")
        root.backward(g)
        torch.cuda.synchronize()
        grads.append(m._hx_arena.grad.float().clone())
        if disable == "" and model == "mirrored":
            assert not calls, "pool backward should have been fused into the Linear dgrad"
        monkeypatch.setattr(K, "maxpool2d_bwd", real)
    assert not HF._PRESCATTERED
    torch.testing.assert_close(grads[0], grads[1], atol=3e-2 * grads[1].abs().max().item(), rtol=3e-2)


@pytest.mark.parametrize("C,CO,k,H,pad,act,p,pk", [(32, 64, 2, 27, 0, "relu", 0.01, 2), (32, 64, 3, 28, 1, "relu", 0.45, 2),
                                                  (16, 32, 3, 14, 0, 0, 0.0, 2), (64, 128, 2, 9, 0, "relu", 0.0, 2),
                                                  (32, 64, 2, 28, 0, "relu", 0.3, 2),  # odd conv output: floor
                                                  (32, 64, 4, 25, 0, "relu", 0.5, 4),  # E1: 22x22 -> 5x5
                                                  (32, 64, 4, 25, 0, "relu", 0.0, 4), (16, 32, 3, 14, 0, 0, 0.0, 4),
                                                  (32, 128, 3, 19, 1, "relu", 0.2, 4), (64, 16, 2, 9, 0, "relu", 0.0, 4)])
def test_conv_fwd_pool_matches_conv_then_pool(C, CO, k, H, pad, act, p, pk):
    """POOL epilogue of conv_fwd_mfma_k (2x2 and 4x4 windows, floor remainders) == conv kernel followed
    by the max-pool(+dropout) kernel, bitwise, argmax included (ties to the lower tap)."""
    from hops_examples_amd.ops import functional as HF

    torch.manual_seed(1)
    B = 5
    x = torch.randn(B, H, H, C, device=dev).to(bf)
    w = (torch.randn(CO, k, k, C, device=dev) * 0.2).to(bf)
    b = torch.randn(CO, device=dev) * 0.1
    g = K.conv_geom(x.shape, w.shape, (1, 1), (pad, pad), (1, 1))
    assert K.conv_fwd_pool_ok(g, act, pk)
    rng = HF.rng_state(dev)
    yp, am = K.conv2d_fwd_pool(x, w, g, bias=b, act=act, drop_p=p, rng=rng, salt=4242, pk=pk)
    yc = K.conv2d_fwd(x, w, g, bias=b, act=act)
    yr, amr = K.maxpool2d_fwd(yc, (pk, pk), (pk, pk), (0, 0), drop_p=p, rng=rng, salt=4242)
    torch.cuda.synchronize()
    assert yp.shape == yr.shape == (B, g[4] // pk, g[5] // pk, CO)
    torch.testing.assert_close(yp.float(), yr.float(), rtol=0, atol=0)
    if act == "relu":
        # the argmax carries ReLU': 0xFF exactly where the window max is 0
        PH, PW = g[4] // pk, g[5] // pk
        wmax = yc[:, :PH * pk, :PW * pk].float().reshape(B, PH, pk, PW, pk, CO).amax((2, 4))
        assert torch.equal(am == 255, wmax <= 0)
        live = am != 255
        assert torch.equal(am[live], amr[live])
    else:
        assert torch.equal(am, amr)


def _e1_net(fuse: bool):
    """The E1 MNIST CNN (mnist.ipynb:154-164: 4x4 convs, 4x4 pool + dropout, dense + dropout) as hopsx
    modules, conv2 -> pool fused in conv2's epilogue when ``fuse`` (what keras.Sequential sets up)."""
    from hops_examples_amd import nn as hnn

    c1 = hnn.Conv2d(1, 32, 4, activation="relu")
    c1.in_affine = (1.0 / 255.0, 0.0)
    c2 = hnn.Conv2d(32, 64, 4, activation="relu")
    pool = hnn.MaxPool2d(4, dropout=0.5)
    drop = hnn.Dropout(0.5)
    pool.salt, drop.salt = 7919, 2 * 7919
    if fuse:
        c2._pool_next, pool._absorbed = (pool,), True
    return torch.nn.Sequential(c1, c2, pool, hnn.Flatten(), hnn.Linear(1600, 128, activation="relu"), drop,
                               hnn.Linear(128, 10))


@pytest.mark.parametrize("fused_scatter", [True, False])
def test_e1_conv_pool4_grads_match_unfused(monkeypatch, fused_scatter):
    """E1: conv2 + 4x4 pool (+dropout) in one launch, and the floor-window pool backward (22x22 -> 5x5:
    the 2 remainder rows / columns get zero gradient) in the Linear's dgrad epilogue or the separate
    pool backward, against the unfused chain: logits and every gradient."""
    from hops_examples_amd.ops import functional as HF
    from hops_examples_amd.runtime.arena import ParamArena

    res = []
    for fuse in (True, False):
        monkeypatch.setenv("HOPSX_DISABLE", "" if fused_scatter else "pool_scatter")
        HF.seed_device_rng(9, dev)
        torch.manual_seed(0)
        m = _e1_net(fuse).to(dev)
        ParamArena.from_module(m, dev)
        calls = []
        real = K.conv2d_fwd_pool
        monkeypatch.setattr(K, "conv2d_fwd_pool", lambda *a, **kw: calls.append(kw.get("pk")) or real(*a, **kw))
        x = torch.randint(0, 256, (32, 28, 28, 1), dtype=torch.uint8, device=dev)
        t = torch.randint(0, 10, (32,), device=dev)
        out = m(x)
        _, _, _, root, g = HF.loss_and_grad_root(out, t, "sparse_ce")
        root.backward(g)
        torch.cuda.synchronize()
        monkeypatch.setattr(K, "conv2d_fwd_pool", real)
        assert calls == ([4] if fuse else []), calls
        res.append((out.float().clone(), None, m._hx_arena.grad.float().clone()))
    assert not HF._PRESCATTERED
    torch.testing.assert_close(res[0][0], res[1][0], rtol=2e-2, atol=2e-3)
    torch.testing.assert_close(res[0][2], res[1][2], atol=3e-2 * res[1][2].abs().max().item(), rtol=3e-2)
    cos = torch.nn.functional.cosine_similarity(res[0][2].double(), res[1][2].double(), dim=0)
    assert cos > 0.9999, float(cos)


@pytest.mark.parametrize("model", ["mirrored", "fashion"])
def test_conv_pool_model_grads_match_unfused(monkeypatch, model):
    """Models running conv2 -> max-pool(+dropout) as one launch train like the unfused chain."""
    from hops_examples_amd.models import mnist
    from hops_examples_amd.ops import functional as HF
    from hops_examples_amd.runtime.arena import ParamArena

    res = []
    for disable in ("", "conv_pool"):
        monkeypatch.setenv("HOPSX_DISABLE", disable)
        HF.seed_device_rng(9, dev)
        torch.manual_seed(0)
        m = (mnist.MirroredMnistCNN() if model == "mirrored" else mnist.FashionMnistCNN()).to(dev)
        for mod in m.modules():
            if hasattr(mod, "salt"):
                mod.salt = 7919
        ParamArena.from_module(m, dev)
        x = torch.randint(0, 256, (32, 28, 28, 1), dtype=torch.uint8, device=dev)
        t = torch.randint(0, 10, (32,), device=dev)
        out = m(x)
        _, _, _, root, g = HF.loss_and_grad_root(out, t, "sparse_ce")
        root.backward(g)
        torch.cuda.synchronize()
        res.append((out.float().clone(), m._hx_arena.grad.float().clone()))
    assert not HF._PRESCATTERED
    # (the conv+pool outputs themselves match bitwise: test_conv_fwd_pool_matches_conv_then_pool; the logits
    # pass through split-K GEMMs whose fp32 atomics land in a run-dependent order, so two runs of the
    # SAME path can differ by a bf16 ulp)
    torch.testing.assert_close(res[0][0], res[1][0], rtol=2e-2, atol=2e-3)
    torch.testing.assert_close(res[0][1], res[1][1], atol=3e-2 * res[1][1].abs().max().item(), rtol=3e-2)


@pytest.mark.parametrize("B,H,C,CO,k,s", [(16, 32, 16, 16, 3, 1), (16, 16, 32, 32, 3, 1), (128, 16, 32, 32, 3, 1),
                                          (8, 12, 64, 32, 3, 1), (32, 8, 64, 64, 3, 1), (16, 16, 16, 32, 3, 2),
                                          (16, 16, 32, 64, 1, 2), (128, 8, 64, 64, 3, 1)])
def test_conv_bwd_pair_kernel_vs_fp32(B, H, C, CO, k, s):
    """conv_bwd_pair_k alone (dgrad + wgrad in one launch) against fp32 autograd, incl. the
    ResNet-20 stage-2 shape (Kd = 288 -> KS = 9), a batch whose dgrad part fills the chip, and the
    GEMM-dgrad variant (conv_bwd_pair_gemm_k: stride 2, or KH*KW*CO = 576 > 512)."""
    torch.manual_seed(5)
    x = (torch.randn(B, H, H, C, device=dev)).to(torch.bfloat16)
    w = (torch.randn(CO, k, k, C, device=dev) / (k * k * C) ** 0.5).to(torch.bfloat16)
    OH = (H + 2 * (k // 2) - k) // s + 1
    dy = torch.randn(B, OH, OH, CO, device=dev).to(torch.bfloat16)
    g = K.conv_geom(x.shape, w.shape, (s, s), (k // 2, k // 2), (1, 1))
    dw = torch.zeros(CO, k, k, C, device=dev)
    dx = K.conv2d_bwd_pair(dy, w, g, x, dw)
    if dx is False:
        pytest.skip("shape not instantiated")
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, None, s, k // 2)
    gx, gw = torch.autograd.grad(yr, (xr, wr), dy.float().permute(0, 3, 1, 2))
    torch.testing.assert_close(dx.float(), gx.permute(0, 2, 3, 1), rtol=2e-2, atol=2e-2 * gx.abs().max().item())
    torch.testing.assert_close(dw, gw.permute(0, 2, 3, 1), rtol=2e-2, atol=1e-2 * gw.abs().max().item())
