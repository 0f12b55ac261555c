"""Keras front end + maggy (lagom search, median early stopping, LOCO ablation) on CPU.

Reference behaviour: notebooks/ml/Parallel_Experiments/Maggy/maggy-fashion-mnist-example.ipynb
(Searchspace prints, lagom result dict), maggy-ablation-titanic-example.ipynb (LOCO trials)."""
import json

import numpy as np
import pytest


def _toy(n=512, d=6, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, d)).astype(np.float32)
    w = rng.normal(size=d)
    y = (x @ w > 0).astype(np.int64)
    return x, y


def test_keras_fit_learns_on_cpu():
    from hops_examples_amd import keras

    x, y = _toy()
    m = keras.Sequential([keras.layers.Dense(32, activation="relu", input_shape=(6,)),
                          keras.layers.Dense(2, activation="softmax")])
    m.compile(optimizer=keras.optimizers.Adam(0.01), loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    h = m.fit(x, y, batch_size=32, epochs=5, verbose=0)
    assert h.history["accuracy"][-1] > 0.9
    assert h.history["loss"][-1] < h.history["loss"][0]
    p = m.predict(x[:10])
    assert p.shape == (10, 2) and np.allclose(p.sum(1), 1, atol=1e-5)
    loss, acc = m.evaluate(x, y, verbose=0)
    assert acc > 0.9
    assert m.count_params() == 6 * 32 + 32 + 32 * 2 + 2


def test_keras_conv_pool_dropout_fusion_and_summary(capsys):
    from hops_examples_amd import keras

    m = keras.Sequential()
    m.add(keras.layers.Conv2D(8, (3, 3), activation="relu", input_shape=(12, 12, 1)))
    m.add(keras.layers.MaxPooling2D((2, 2)))
    m.add(keras.layers.Dropout(0.25))
    m.add(keras.layers.Flatten())
    m.add(keras.layers.Dense(10, activation="softmax", name="out"))
    m.build()
    pools = [mod for mod in m.net.modules() if type(mod).__name__ == "MaxPool2d"]
    assert pools and pools[0].dropout == 0.25  # pool + dropout fused into one kernel
    m.summary()
    out = capsys.readouterr().out
    assert "Total params: " in out and "out (Dense)" in out
    assert m.get_layer("out").output_shape == (None, 10)


def test_keras_callbacks_and_checkpoint(tmp_path):
    from hops_examples_amd import keras

    x, y = _toy(256)
    seen = []

    class CB(keras.callbacks.Callback):
        def on_batch_end(self, batch, logs=None):
            seen.append(logs["loss"])

    m = keras.Sequential([keras.layers.Dense(8, activation="relu", input_shape=(6,)),
                          keras.layers.Dense(2, activation="softmax")])
    m.compile("adam", "sparse_categorical_crossentropy", ["accuracy"])
    ck = tmp_path / "w.pt"
    m.fit(x, y, batch_size=64, epochs=2, verbose=0, callbacks=[CB(), keras.callbacks.ModelCheckpoint(ck, "loss")],
          validation_data=(x, y))
    assert len(seen) == 8 and ck.exists()
    m2 = keras.Sequential([keras.layers.Dense(8, activation="relu", input_shape=(6,)),
                           keras.layers.Dense(2, activation="softmax")])
    m2.build()
    m2.load_weights(ck)
    np.testing.assert_allclose(m2.predict(x[:4]), m.predict(x[:4]), atol=1e-6)


def test_searchspace_prints_and_samples(capsys):
    from hops_examples_amd.maggy import Searchspace

    sp = Searchspace(kernel=("INTEGER", [2, 8]), pool=("INTEGER", [2, 8]))
    sp.add("dropout", ("DOUBLE", [0.01, 0.99]))
    out = capsys.readouterr().out
    assert out.splitlines() == ["Hyperparameter added: kernel", "Hyperparameter added: pool",
                                "Hyperparameter added: dropout"]
    import random

    s = sp.sample(random.Random(0))
    assert 2 <= s["kernel"] <= 8 and 0.01 <= s["dropout"] <= 0.99
    with pytest.raises(ValueError):
        sp.add("bad", ("FLOAT", [0, 1]))


def test_lagom_randomsearch_and_early_stop(project_root, monkeypatch):
    from hops_examples_amd.maggy import Searchspace, lagom

    monkeypatch.setenv("HOPSX_NUM_GPUS", "0")
    sp = Searchspace(x=("DOUBLE", [0.0, 1.0]))

    def train_fn(x, reporter):
        import time

        # trials with small x are "bad" and slow: the median rule should stop some of them
        for step in range(40):
            reporter.broadcast(metric=x, step=step)
            time.sleep(0.01 if x > 0.5 else 0.05)
        return x

    res = lagom(train_fn, sp, optimizer="randomsearch", direction="max", num_trials=6, name="t",
                hb_interval=0.05, es_interval=0.1, es_min=2, seed=3)
    assert res["num_trials"] == 6
    assert res["best_val"] == max(res["metric_list"])
    assert 0 <= res["best_hp"]["x"] <= 1
    exp = sorted((project_root / "Experiments").iterdir())[-1]
    data = json.loads((exp / "result.json").read_text())
    assert len(data["trials"]) == 6


def test_lagom_gridsearch_min(project_root, monkeypatch):
    from hops_examples_amd.maggy import Searchspace, lagom

    monkeypatch.setenv("HOPSX_NUM_GPUS", "0")
    sp = Searchspace(a=("DISCRETE", [1, 2, 3]), b=("CATEGORICAL", ["u", "v"]))

    def train_fn(a, b, reporter):
        reporter.broadcast(a + (0.5 if b == "v" else 0))
        return {"metric": a + (0.5 if b == "v" else 0)}

    res = lagom(train_fn, sp, optimizer="gridsearch", direction="min", num_trials=0, es_interval=1e9)
    assert res["num_trials"] == 6 and res["best_val"] == 1 and res["best_hp"] == {"a": 1, "b": "u"}


def test_ablation_loco_trials(project_root, monkeypatch):
    from hops_examples_amd import keras
    from hops_examples_amd.maggy import AblationStudy, lagom
    from hops_examples_amd.maggy.ablation import trial_generators

    monkeypatch.setenv("HOPSX_NUM_GPUS", "0")
    st = AblationStudy("titanic_train_dataset", 1, label_name="survived")
    st.features.include("pclass")
    st.features.include(["fare", "sibsp"])

    def base():
        from hops_examples_amd import keras as K

        m = K.Sequential()
        m.add(K.layers.Dense(16, activation="relu"))
        m.add(K.layers.Dense(16, name="my_dense_two", activation="relu"))
        m.add(K.layers.Dense(8, name="my_dense_three", activation="relu"))
        m.add(K.layers.Dense(2, activation="softmax", name="head"))
        return m

    st.model.set_base_model_generator(base)
    st.model.layers.include("my_dense_two", "my_dense_three")
    st.model.layers.include_groups(prefix="my_dense")

    def gen(ablated, epochs, batch):
        import numpy as np

        rng = np.random.default_rng(0)
        allc = ["pclass", "fare", "sibsp", "age"]
        full = rng.normal(size=(256, 4)).astype(np.float32)
        y = (full[:, 0] > 0).astype(np.int64)
        x = full[:, [i for i, c in enumerate(allc) if c != ablated]]
        for _ in range(epochs):
            for s in range(0, 256, batch):
                yield x[s:s + batch], y[s:s + batch]

    st.set_dataset_generator(gen)
    trials = trial_generators(st)
    names = [t for t, _ in trials]
    assert names == ["base", "feature-pclass", "feature-fare", "feature-sibsp", "layer-my_dense_two",
                     "layer-my_dense_three", "layers-prefix-my_dense"]
    m = dict(trials)["layers-prefix-my_dense"]["model_function"]()
    assert [l.name for l in m.layers] == [m.layers[0].name, "head"]

    def training_fn(dataset_function, model_function):
        from hops_examples_amd import keras as K

        model = model_function()
        model.compile(optimizer=K.optimizers.Adam(0.01), loss="sparse_categorical_crossentropy",
                      metrics=["accuracy"])
        h = model.fit(dataset_function(3, 32), epochs=3, steps_per_epoch=8, verbose=0)
        return float(h.history["accuracy"][-1])

    res = lagom(training_fn, experiment_type="ablation", ablation_study=st, ablator="loco", name="Titanic-LOCO")
    assert set(res["results"]) == set(names)
    assert res["results"]["base"] > 0.8
    # removing the only informative feature hurts
    assert res["results"]["feature-pclass"] < res["results"]["base"]


def _flagship_keras(keras, dense_act="softmax"):
    """The reference's MirroredStrategy MNIST model, written the notebook's way
    (mirroredstrategy_mnist_example.ipynb:189-207)."""
    return keras.Sequential([
        keras.layers.Conv2D(32, 2, activation="relu", input_shape=(28, 28, 1)),
        keras.layers.Conv2D(64, 2, activation="relu"),
        keras.layers.MaxPooling2D(),
        keras.layers.Dropout(0.01),
        keras.layers.Flatten(),
        keras.layers.Dense(128, activation="relu"),
        keras.layers.Dense(10, activation=dense_act),
    ])


def test_keras_flagship_stack_matches_the_persistent_engine_structurally():
    """fit's resident-epoch path can run the persistent engine only on the reference model's exact layer
    stack (runtime.persist.flagship_layers over a view of the Keras modules); uint8 pixels go straight
    into the first conv, which normalises them itself (same values as the separate x / 255 pass)."""
    import torch

    from hops_examples_amd import keras
    from hops_examples_amd.runtime.persist import flagship_layers

    m = _flagship_keras(keras)
    m.build()
    v = m._flagship_view()
    assert v is not None and flagship_layers(v) is not None
    assert v.conv1.in_affine == (1.0 / 255.0, 0.0) and v.fc2.weight.shape == (10, 128)
    from hops_examples_amd import nn as hnn

    lins = [mod for mod in m.net.modules() if isinstance(mod, hnn.Linear)]
    assert v.fc1 is lins[0] and v.fc2 is lins[1]  # the view shares the Keras model's layers (and parameters)
    for other in (
        keras.Sequential([keras.layers.Conv2D(32, 3, activation="relu", input_shape=(28, 28, 1)),
                          keras.layers.Conv2D(64, 2, activation="relu"), keras.layers.MaxPooling2D(),
                          keras.layers.Flatten(), keras.layers.Dense(128, activation="relu"),
                          keras.layers.Dense(10, activation="softmax")]),  # k3 first conv
        keras.Sequential([keras.layers.Dense(64, activation="relu", input_shape=(784,)),
                          keras.layers.Dense(10, activation="softmax")]),
    ):
        other.build()
        assert other._flagship_view() is None
    # raw uint8 into conv1 (in_affine) == the normalised float input
    x8 = torch.randint(0, 256, (2, 28, 28, 1), dtype=torch.uint8)
    m.eval()
    a = m(x8)
    b = m.net[1:](x8.float() / 255.0)
    torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
