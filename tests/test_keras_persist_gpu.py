"""keras.Sequential.fit on the reference's MirroredStrategy MNIST model (mirroredstrategy_mnist_example.ipynb:
189-231: the notebook's layer stack, Adadelta, sparse CE, batch 32) takes the persistent whole-step engine
through the resident-epoch path (keras.py _fit_epoch_fast): same training as the multi-kernel TrainStep fit,
at the persistent engine's speed."""
import os
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)


def _model(keras):
    return keras.Sequential([
        keras.layers.Conv2D(32, 2, activation="relu", input_shape=(28, 28, 1)),
        keras.layers.Conv2D(64, 2, activation="relu"),
        keras.layers.MaxPooling2D(),
        keras.layers.Dropout(0.01),
        keras.layers.Flatten(),
        keras.layers.Dense(128, activation="relu"),
        keras.layers.Dense(10, activation="softmax"),
    ])


def _data(n, seed=0):
    rng = np.random.default_rng(seed)
    y = rng.integers(0, 10, n)
    x = rng.integers(0, 60, (n, 28, 28, 1)).astype(np.uint8)
    for c in range(10):  # a learnable signal: a bright class-dependent stripe
        x[y == c, 2 * c + 3: 2 * c + 5, 4:24, 0] = 230
    return x, y.astype(np.int64)


def _fit(persist: bool, x, y, epochs=2):
    from hops_examples_amd import keras

    old = os.environ.get("HOPSX_PERSIST")
    os.environ["HOPSX_PERSIST"] = "1" if persist else "0"
    try:
        torch.manual_seed(0)
        m = _model(keras)
        m.compile(optimizer=keras.optimizers.Adadelta(1.0), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy"])
        h = m.fit(x, y, batch_size=32, epochs=epochs, verbose=0, shuffle=True, seed=3)
        return m, h
    finally:
        if old is None:
            os.environ.pop("HOPSX_PERSIST", None)
        else:
            os.environ["HOPSX_PERSIST"] = old


def test_keras_fit_runs_the_persistent_engine_and_learns():
    x, y = _data(4096 + 17)  # + a partial last batch (TrainStep)
    m, h = _fit(True, x, y)
    assert m._fast is not None and m._fast.kind == "persistent", "fit did not take the persistent engine"
    m._fast.check()
    acc = h.history["accuracy"]
    assert h.history["loss"][-1] < h.history["loss"][0] and acc[-1] > 0.9, h.history
    m2, h2 = _fit(False, x, y)
    assert m2._fast is None
    # same model, optimizer and data order: the two engines train alike (bf16 numerics differ in detail)
    assert abs(h2.history["accuracy"][-1] - acc[-1]) < 0.05, (h.history, h2.history)
    loss, a = m.evaluate(x[:1024], y[:1024], verbose=0)
    assert a > 0.9


def test_keras_fit_persistent_throughput():
    """60k-image epochs through keras fit: images/s printed (the resident-epoch path launches 32 steps at a
    time, so fit runs near the engine's own rate)."""
    x, y = _data(60000, seed=1)
    m, _ = _fit(True, x, y, epochs=1)  # warm-up epoch (upload, first launches)
    t = time.perf_counter()
    m.fit(x, y, batch_size=32, epochs=2, verbose=0)
    torch.cuda.synchronize()
    ips = 2 * 60000 / (time.perf_counter() - t)
    print(f"keras fit on the persistent engine: {ips:,.0f} images/s")
    assert m._fast is not None and ips > 3e5, ips


def test_keras_fit_resident_e1_model():
    """Any model fit on whole arrays (here the E1 Keras MNIST CNN, mnist.ipynb:154-164: k4 convs, pool 4,
    dropout, Adam) trains on device-resident data: by default the TrainStep's multi-step graphs over a
    resident epoch buffer (keras.py _fit_epoch_resident); HOPSX_KERAS_RESIDENT=0 gathers per batch on the
    device; HOPSX_KERAS_DEVICE_BATCHES=0 copies every batch from the host.  All learn alike; images/s printed."""
    from hops_examples_amd import keras

    x, y = _data(8192 + 5, seed=2)  # + a partial last batch
    modes = {"resident": {}, "device_batches": {"HOPSX_KERAS_RESIDENT": "0"},
             "host_batches": {"HOPSX_KERAS_RESIDENT": "0", "HOPSX_KERAS_DEVICE_BATCHES": "0"}}
    res = {}
    for name, env in modes.items():
        os.environ.update(env)
        try:
            torch.manual_seed(0)
            m = keras.Sequential([
                keras.layers.Conv2D(32, 4, activation="relu", input_shape=(28, 28, 1)),
                keras.layers.Conv2D(64, 4, activation="relu"),
                keras.layers.MaxPooling2D(4),
                keras.layers.Dropout(0.5),
                keras.layers.Flatten(),
                keras.layers.Dense(128, activation="relu"),
                keras.layers.Dropout(0.5),
                keras.layers.Dense(10, activation="softmax"),
            ])
            m.compile(optimizer="adam", loss="sparse_categorical_crossentropy", metrics=["accuracy"])
            h0 = m.fit(x, y, batch_size=32, epochs=1, verbose=0)  # warm-up epoch (build, graph capture)
            torch.cuda.synchronize()
            t = time.perf_counter()
            h = m.fit(x, y, batch_size=32, epochs=2, verbose=0)
            torch.cuda.synchronize()
            res[name] = (round(2 * len(x) / (time.perf_counter() - t)), h0.history["loss"][0],
                         h.history["loss"][-1], h.history["accuracy"][-1])
        finally:
            for k in env:
                os.environ.pop(k, None)
    print("keras fit E1 model (images/s, first-epoch loss, last loss, last accuracy):", res)
    for name, (_, l0, l1, acc) in res.items():
        assert acc > 0.9 and l1 < l0, (name, res)
    # the first epoch sees the same data in the same order in every mode: its mean loss agrees
    assert abs(res["resident"][1] - res["host_batches"][1]) < 0.1 * res["host_batches"][1] + 0.05, res
