"""GPU checks for the wide & deep taxi model, fixed-length embedding bags, sliced
optimizers and the Keras front end (numerics vs the fp32 CPU path)."""
import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from hops_examples_amd.models import widedeep as W  # noqa: E402
from hops_examples_amd.ops import functional as HF  # noqa: E402
from hops_examples_amd.ops import kernels as K  # noqa: E402
from hops_examples_amd.runtime.arena import ParamArena  # noqa: E402
from hops_examples_amd.runtime.step import TrainStep  # noqa: E402


@pytest.mark.parametrize("dim,L,mode", [(1, 13, 0), (8, 5, 1), (40, 3, 0)])
def test_embedding_bag_fixed_length(dim, L, mode):
    torch.manual_seed(0)
    V, B = 300, 97
    table = torch.randn(V, dim, device="cuda")
    idx = torch.randint(0, V, (B, L), device="cuda")
    out = torch.empty(B, dim, device="cuda")
    K.embedding_bag_fwd(table, idx.reshape(-1), None, mode, out, bag_len=L)
    ref = table[idx].sum(1) if mode == 0 else table[idx].mean(1)
    torch.testing.assert_close(out, ref, atol=1e-4, rtol=1e-4)
    dout = torch.randn(B, dim, device="cuda")
    dt = torch.zeros(V, dim, device="cuda")
    K.embedding_bag_bwd(dout, idx.reshape(-1), None, mode, dt, B, bag_len=L)
    t2 = table.clone().requires_grad_(True)
    r = t2[idx].sum(1) if mode == 0 else t2[idx].mean(1)
    r.backward(dout)
    torch.testing.assert_close(dt, t2.grad, atol=1e-4, rtol=1e-4)


def test_widedeep_grads_match_cpu():
    torch.manual_seed(0)
    cpu = W.TaxiWideDeep()
    with torch.no_grad():
        cpu.wide.weight.normal_(0, 0.1)
    gpu = copy.deepcopy(cpu).cuda()
    ParamArena.from_module(gpu)
    ParamArena.from_module(cpu)
    d, c, y = W.synth_taxi(256, seed=3)
    lc = HF.loss(cpu(d, c), y, "bce_logits")
    lc.backward()
    lg = HF.loss(gpu(d.cuda(), c.cuda()), y.cuda(), "bce_logits")
    lg.backward()
    assert abs(lc.item() - lg.item()) < 0.02
    gc, gg = cpu._hx_arena.grad.double(), gpu._hx_arena.grad.cpu().double()
    cos = torch.nn.functional.cosine_similarity(gc, gg, dim=0).item()
    assert cos > 0.99, cos


def test_widedeep_graph_training_and_sliced_optimizers():
    torch.manual_seed(0)
    m = W.TaxiWideDeep().cuda()
    ParamArena.from_module(m)
    opt = W.make_optimizer(m)
    a = m._hx_arena
    assert opt.opts[0]._sl.stop == opt.opts[1]._sl.start
    st = TrainStep(m, opt, "bce_logits", graph=True, forward_fn=lambda mm, x: mm(*x))
    d, c, y = W.synth_taxi(40 * 500, seed=5, device="cuda")
    d = d.to(torch.bfloat16)
    losses = []
    for ep in range(3):
        tot = torch.zeros((), device="cuda")
        for i in range(500):
            s = slice(i * 40, (i + 1) * 40)
            r = st((d[s], c[s]), y[s])
            tot += r["loss"].reshape(-1)[0]
        losses.append(tot.item() / 500)
    assert all(np.isfinite(losses)) and losses[-1] < losses[0] - 0.02, losses
    assert float(opt.opts[0].step_count) == 1500 and float(opt.opts[1].step_count) == 1500
    assert a.grad.abs().max().item() == 0.0  # the fused optimizers zero their slices


def test_keras_fit_on_gpu():
    from hops_examples_amd import keras

    rng = np.random.default_rng(0)
    x = rng.integers(0, 128, (2048, 28, 28, 1), dtype=np.uint8)
    y = rng.integers(0, 2, 2048)
    x[y == 1, 2:10, 2:10] += 120  # class 1: bright top-left patch, class 0: bright bottom-right patch
    x[y == 0, 18:26, 18:26] += 120
    m = keras.Sequential([
        keras.layers.Conv2D(16, (3, 3), activation="relu", input_shape=(28, 28, 1)),
        keras.layers.MaxPooling2D((2, 2)),
        keras.layers.Flatten(),
        keras.layers.Dense(32, activation="relu"),
        keras.layers.Dense(2, activation="softmax"),
    ])
    m.compile(keras.optimizers.Adam(0.003), "sparse_categorical_crossentropy", ["accuracy"])
    h = m.fit(x, y, batch_size=64, epochs=4, verbose=0)
    assert m.device.type == "cuda"
    assert h.history["accuracy"][-1] > 0.85, h.history
    p = m.predict(x[:8])
    assert p.shape == (8, 2) and np.allclose(p.sum(1), 1, atol=1e-3)
