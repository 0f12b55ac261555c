"""Model zoo on CPU: parameter counts vs the reference notebooks (SURVEY Appendix models
table), wide & deep / census linear learn, optimizer slices over one arena."""
import numpy as np
import pandas as pd
import pytest
import torch


@pytest.mark.parametrize("name,count", [("simulated_mlp", 193), ("titanic_dnn", 7813), ("mnist_mlp", 101770),
                                        ("keras_mnist_cnn", 239594), ("fashion_mnist_cnn", 1625866)])
def test_zoo_param_counts(name, count):
    from hops_examples_amd.models import zoo

    m = getattr(zoo, name)()
    m.build()
    assert m.count_params() == count


def test_resnet_param_counts_and_forward():
    from hops_examples_amd.models import resnet

    assert sum(p.numel() for p in resnet.resnet50().parameters()) == 25_557_032
    m = resnet.cifar_resnet(20)
    assert sum(p.numel() for p in m.parameters()) == 272_474
    y = m(torch.randint(0, 256, (2, 32, 32, 3), dtype=torch.uint8))
    assert y.shape == (2, 10) and torch.isfinite(y).all()


def test_widedeep_learns_with_sliced_optimizers():
    from hops_examples_amd.models import widedeep as W
    from hops_examples_amd.runtime.arena import ParamArena
    from hops_examples_amd.runtime.step import TrainStep

    assert W.WIDE_ROWS == 6287 and W.hidden_units() == [100, 70, 48, 34]
    torch.manual_seed(0)
    m = W.TaxiWideDeep()
    ParamArena.from_module(m)
    opt = W.make_optimizer(m)
    a, b = opt.opts[0]._sl, opt.opts[1]._sl
    assert a.start == 0 and a.stop == b.start and b.stop == m._hx_arena.numel
    st = TrainStep(m, opt, "bce_logits", graph=False, forward_fn=lambda mm, x: mm(*x))
    d, c, y = W.synth_taxi(40 * 300, seed=1)
    ls = []
    for ep in range(2):
        tot = 0.0
        for i in range(300):
            s = slice(i * 40, (i + 1) * 40)
            tot += float(st((d[s], c[s]), y[s])["loss"])
        ls.append(tot / 300)
    assert ls[1] < ls[0] < 0.7
    assert float(opt.opts[0].step_count) == 600


def test_optimizer_subset_must_be_contiguous():
    from hops_examples_amd import optim
    from hops_examples_amd.runtime.arena import ParamArena

    m = torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.Linear(4, 4), torch.nn.Linear(4, 4))
    ParamArena.from_module(m)
    optim.SGD(m[1], lr=0.1)  # a sub-module is fine
    with pytest.raises(ValueError):
        optim.SGD([m[0].weight, m[2].weight], lr=0.1)


def test_census_linear_classifier():
    from hops_examples_amd.models.linear import LinearClassifier

    rng = np.random.default_rng(0)
    n = 3000
    df = pd.DataFrame({"Age": rng.integers(18, 80, n), "Sex": rng.choice(["Male", "Female"], n)})
    logit = 0.06 * (df.Age - 45) + np.where(df.Sex == "Male", 1.0, -1.0)
    df["Over-50K"] = (rng.random(n) < 1 / (1 + np.exp(-logit))).astype(np.int64)
    m = LinearClassifier(["Age"], {"Sex": ["Male", "Female"]})
    m.fit(df, "Over-50K", steps=800, device="cpu")
    ev = m.evaluate(df, "Over-50K")
    assert ev["accuracy"] > 0.7
    p = m.predict_proba(pd.DataFrame({"Age": [50, 50], "Sex": ["Male", "Female"]}))
    assert p[0] > p[1]  # what-if: flipping Sex changes the prediction in the learned direction
    p_oov = m.predict_proba(pd.DataFrame({"Age": [50], "Sex": ["unknown"]}))
    assert 0 < p_oov[0] < 1
