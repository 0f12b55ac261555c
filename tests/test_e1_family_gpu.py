"""The E1 / E8 / E9 / E11 model family (mnist.ipynb:154-164, grid_search_fashion_mnist.ipynb:224-227,
evolutionary_search_mnist.ipynb:264, maggy-fashion-mnist-example.ipynb:188-327): Conv2D(32, k) -> Conv2D(64, k)
-> MaxPooling2D(p) -> Dropout -> Flatten -> Dense(128) -> Dropout -> Dense(10), with the kernel and pool size as
the searched hyper-parameters (maggy's Searchspace: kernel and pool in [2, 8]).

One training step per (kernel, pool) pair on the kernels, as keras.Sequential wires the layers (conv2 + pool in
one launch where the pool is 2x2 / 4x4, the rest unfused), against fp64 PyTorch on the same bf16 weights with
the activations and their gradients rounded to bf16 where the kernels store them: the logits, and every
parameter's gradient per tensor (cos >= 0.995, see the test), and every op's forward on the kernels' own inputs
(cos >= 0.99999).  Dropout off (its masks are pinned by the
fused-vs-unfused tests); batch 32 and the E11 batch of 512."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd import nn as hnn  # noqa: E402
from hops_examples_amd.ops import functional as HF  # noqa: E402
from hops_examples_amd.runtime.arena import ParamArena  # noqa: E402

dev = torch.device("cuda", 0)


def _net(k, p):
    c1 = hnn.Conv2d(1, 32, k, activation="relu")
    c1.in_affine = (1.0 / 255.0, 0.0)
    c2 = hnn.Conv2d(32, 64, k, activation="relu")
    pool = hnn.MaxPool2d(p, dropout=0.0)
    c2._pool_next, pool._absorbed = (pool,), True  # as keras.Sequential.build wires Conv2D -> MaxPooling2D
    s = (30 - 2 * k) // p
    return torch.nn.Sequential(c1, c2, pool, hnn.Flatten(), hnn.Linear(s * s * 64, 128, activation="relu"),
                               hnn.Linear(128, 10))


def _reference(m, x_u8, y):
    """fp64 NCHW PyTorch of the same network on the bf16 weights the kernels read."""
    from hops_examples_amd.runtime.persist import _RoundFwd, _RoundGrad

    def bf(t):  # a bf16-stored activation: value rounded, and its gradient rounded where the backward stores it
        return _RoundGrad.apply(_RoundFwd.apply(t))

    P = {n: p.detach().cpu().to(torch.bfloat16).double().clone().requires_grad_(True) for n, p in m.named_parameters()}
    pool = m[2]
    x = x_u8.double().permute(0, 3, 1, 2) / 255.0
    h = bf(F.relu(F.conv2d(x, P["0.weight"].permute(0, 3, 1, 2), P["0.bias"])))
    h = bf(F.relu(F.conv2d(h, P["1.weight"].permute(0, 3, 1, 2), P["1.bias"])))
    h = bf(F.max_pool2d(h, pool.k))
    h = h.permute(0, 2, 3, 1).reshape(h.shape[0], -1)  # NHWC flatten, as the kernels lay it out
    h = bf(F.relu(h @ P["4.weight"].t() + P["4.bias"]))
    logits = h @ P["5.weight"].t() + P["5.bias"]
    F.cross_entropy(logits, y).backward()
    return logits.detach(), {n: t.grad for n, t in P.items()}


@pytest.mark.parametrize("k,p,B", [(2, 2, 32), (3, 2, 32), (4, 4, 32), (5, 3, 32), (3, 4, 32), (2, 8, 32),
                                   (8, 2, 32), (6, 5, 32), (4, 4, 512), (3, 2, 512)])
def test_e1_family_step_vs_fp64(k, p, B):
    torch.manual_seed(k * 10 + p)
    m = _net(k, p).to(dev)
    ParamArena.from_module(m, dev)
    x = torch.randint(0, 256, (B, 28, 28, 1), dtype=torch.uint8, device=dev)
    y = torch.randint(0, 10, (B,), device=dev)
    out = m(x)
    _, _, _, root, g = HF.loss_and_grad_root(out, y, "sparse_ce")
    root.backward(g)
    torch.cuda.synchronize()
    ref_logits, ref = _reference(m, x.cpu(), y.cpu())
    lg = out.detach().double().cpu()
    cos_l = F.cosine_similarity(lg.flatten(), ref_logits.flatten(), dim=0)
    assert cos_l > 0.9999, float(cos_l)
    bad = []
    for n, prm in m.named_parameters():
        gk = prm.grad.double().cpu().flatten()
        gr = ref[n].flatten()
        c = float(F.cosine_similarity(gk, gr, dim=0))
        rel = float((gk - gr).norm() / gr.norm().clamp_min(1e-30))
        # (0.995: a conv2 output one bf16 ulp apart between the fp32-accumulated kernel and fp64 flips a
        # max-pool argmax or a ReLU; with 5x5+ kernels (K >= 800) that moves the conv gradients to ~0.996,
        # while every op's own output matches fp64 to 0.99999 below)
        if c < 0.995 or rel > 0.1:
            bad.append((n, c, rel))
    assert not bad, (k, p, B, bad)
    # every op's forward on the kernels' own inputs (teacher-forced): conv1, conv2, pool, dense
    W = {n: prm.detach().cpu().to(torch.bfloat16).double() for n, prm in m.named_parameters()}

    def cos(a, b):
        return float(F.cosine_similarity(a.double().cpu().flatten(), b.double().cpu().flatten(), dim=0))

    with torch.no_grad():
        y1 = m[0](x)
        r1 = F.relu(F.conv2d(x.cpu().double().permute(0, 3, 1, 2) / 255.0, W["0.weight"].permute(0, 3, 1, 2),
                             W["0.bias"]))
        y2 = m[1].conv_only(y1)
        r2 = F.relu(F.conv2d(y1.cpu().double().permute(0, 3, 1, 2), W["1.weight"].permute(0, 3, 1, 2), W["1.bias"]))
        yp = m[1](y1)  # conv2 + pool as the step runs it (one launch for 2x2 / 4x4)
        rp = F.max_pool2d(y2.cpu().double().permute(0, 3, 1, 2), p)
        h = m[4](yp.reshape(B, -1))
        rh = F.relu(yp.cpu().double().reshape(B, -1) @ W["4.weight"].t() + W["4.bias"])
    for name, a, r in (("conv1", y1, r1.permute(0, 2, 3, 1)), ("conv2", y2, r2.permute(0, 2, 3, 1)),
                       ("pool", yp, rp.permute(0, 2, 3, 1)), ("dense1", h, rh)):
        assert cos(a, r) > 0.99999, (name, k, p, B, cos(a, r))
