"""Input layer fused into the next conv's operand gather (conv_mfma.hip IN0): pool(conv(conv0(x)))
in one launch.  The fused launch must reproduce the unfused chain bit for bit (same fp32 order in
the input layer, same bf16 roundings) and the chain must match an fp32 PyTorch reference."""
import math
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd.ops import kernels as K  # noqa: E402

dev = "cuda"
bf = torch.bfloat16


def _nchw_conv(x, w, b, pad):
    return F.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), b, 1, pad).permute(0, 2, 3, 1)


@pytest.mark.parametrize("B,HW,k0,k,pad,drop", [
    (32, 28, 2, 2, 0, 0.0),    # MirroredMnistCNN conv1 -> conv2 -> pool (bench config)
    (32, 28, 2, 2, 0, 0.01),   # ... with its fused Dropout(0.01)
    (7, 28, 3, 3, 1, 0.0),     # FashionMnistCNN ('same' 3x3 convs), odd batch
    (5, 21, 2, 3, 1, 0.0),     # mixed kernel sizes
])
def test_conv_in_pool_matches_unfused_and_fp32(B, HW, k0, k, pad, drop):
    torch.manual_seed(0)
    C, CO = 32, 64
    scale, shift = 1.0 / 255.0, -0.5
    x = torch.randint(0, 256, (B, HW, HW, 1), dtype=torch.uint8, device=dev)
    w0 = (torch.randn(C, k0, k0, 1, device=dev) / math.sqrt(k0 * k0)).to(bf)
    b0 = torch.randn(C, device=dev) * 0.1
    w = (torch.randn(CO, k, k, C, device=dev) / math.sqrt(k * k * C)).to(bf)
    b = torch.randn(CO, device=dev) * 0.1
    p0 = 0 if k0 == 2 else pad
    g0 = K.conv_geom(x.shape, w0.shape, (1, 1), (p0, p0), (1, 1))
    g = K.conv_geom((B, g0[4], g0[5], C), w.shape, (1, 1), (pad, pad), (1, 1))
    assert K.conv_fwd_pool_in_ok(g0, g, "relu")
    rng = torch.tensor([1234, 7], dtype=torch.int64, device=dev)
    y, am, y1 = K.conv2d_fwd_pool_in(x, w0, b0, "relu", g0, w, g, bias=b, act="relu", drop_p=drop, rng=rng,
                                     salt=99, in_affine=(scale, shift))
    # unfused chain: direct input-layer kernel, then conv + pool launch
    y1_ref = K.conv2d_fwd(x, w0, g0, bias=b0, act="relu", in_affine=(scale, shift))
    y_ref, am_ref = K.conv2d_fwd_pool(y1_ref, w, g, bias=b, act="relu", drop_p=drop, rng=rng, salt=99)
    torch.cuda.synchronize()
    assert torch.equal(y1.view(torch.int16), y1_ref.view(torch.int16))
    assert torch.equal(y.view(torch.int16), y_ref.view(torch.int16))
    assert torch.equal(am, am_ref)
    if drop == 0.0:
        # fp32 reference of the chain (input layer rounded to bf16 as it is stored)
        xf = x.float() * scale + shift
        r1 = _nchw_conv(xf, w0.float(), b0, p0).relu().to(bf).float()
        r2 = _nchw_conv(r1, w.float(), b, pad).relu()
        ref = F.max_pool2d(r2.permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)
        err = (y.float() - ref).abs().max().item()
        assert err <= 1e-2 * ref.abs().max().item() + 1e-3, err
    # inference form: the input layer's output is not kept
    y2, _, none = K.conv2d_fwd_pool_in(x, w0, b0, "relu", g0, w, g, bias=b, act="relu", drop_p=drop, rng=rng,
                                       salt=99, in_affine=(scale, shift), keep_y1=False)
    assert none is None and torch.equal(y2.view(torch.int16), y.view(torch.int16))


def _train_step_grads(fused: bool):
    from hops_examples_amd.models.mnist import MirroredMnistCNN
    from hops_examples_amd.ops import functional as HF
    from hops_examples_amd.runtime.arena import ParamArena

    old = os.environ.get("HOPSX_CONV_IN_POOL")
    os.environ["HOPSX_CONV_IN_POOL"] = "1" if fused else "0"  # opt-in path (off by default)
    try:
        torch.manual_seed(3)
        m = MirroredMnistCNN().to(dev)
        m.pool.salt = 4242  # dropout masks: the salt counter differs between model instances
        ParamArena.from_module(m, dev)
        x = torch.randint(0, 256, (32, 28, 28, 1), dtype=torch.uint8, device=dev)
        yl = torch.randint(0, 10, (32,), device=dev)
        out = m(x)
        loss, _, _, dl = HF.loss_and_grad(out, yl, "sparse_ce")
        out.backward(dl)
        torch.cuda.synchronize()
        return out.float().clone(), m._hx_arena.grad.clone()
    finally:
        if old is None:
            os.environ.pop("HOPSX_CONV_IN_POOL", None)
        else:
            os.environ["HOPSX_CONV_IN_POOL"] = old


def test_mirrored_mnist_fused_input_layer_same_step():
    """The flagship model's step with the fused input layer equals the unfused one (up to the order
    of fp32 atomic accumulation downstream)."""
    out_f, g_f = _train_step_grads(True)
    out_u, g_u = _train_step_grads(False)
    # the conv chain is bit-identical (test above); fc1's split-K forward and the weight gradients
    # accumulate with fp32 atomics in run-dependent order, so the rest agrees to rounding noise
    assert (out_f - out_u).abs().max().item() <= 1e-2 * out_u.abs().max().item()
    err = (g_f - g_u).abs().max().item()
    assert err <= 2e-2 * g_u.abs().max().item(), err
    assert g_f.abs().sum() > 0
