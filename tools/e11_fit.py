"""keras fit throughput of the E1-family CNN across the maggy Searchspace's kernel / pool sizes
(maggy-fashion-mnist-example.ipynb:121-127, 188-327: Conv2D(32,k) Conv2D(64,k) MaxPooling2D(p) Dropout Dense(128)
Dropout Dense(10), Adam, batch 512 in E11; batch 32 in E1), synthetic uint8 data.  One JSON line per config."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hops_examples_amd import keras  # noqa: E402

rng = np.random.default_rng(0)
n = 16384
x = rng.integers(0, 255, (n, 28, 28, 1)).astype(np.uint8)
y = rng.integers(0, 10, n)
for bs, k, p in [(512, 2, 2), (512, 3, 2), (512, 4, 4), (512, 5, 3), (512, 8, 2), (512, 3, 8), (32, 4, 4), (32, 3, 2)]:
    torch.manual_seed(0)
    m = keras.Sequential([
        keras.layers.Conv2D(32, k, activation="relu", input_shape=(28, 28, 1)),
        keras.layers.Conv2D(64, k, activation="relu"),
        keras.layers.MaxPooling2D(p),
        keras.layers.Dropout(0.3),
        keras.layers.Flatten(),
        keras.layers.Dense(128, activation="relu"),
        keras.layers.Dropout(0.3),
        keras.layers.Dense(10, activation="softmax"),
    ])
    m.compile(optimizer="adam", loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    m.fit(x, y, batch_size=bs, epochs=1, verbose=0)  # build, capture
    torch.cuda.synchronize()
    t = time.perf_counter()
    h = m.fit(x, y, batch_size=bs, epochs=2, verbose=0)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    print(json.dumps({"batch": bs, "kernel": k, "pool": p, "images_per_sec": round(2 * n / el),
                      "loss": round(h.history["loss"][-1], 4)}), flush=True)
