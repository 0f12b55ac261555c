"""keras fit of the E1 MNIST CNN (mnist.ipynb:154-164) on synthetic uint8 data: for kernel profiling."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hops_examples_amd import keras  # noqa: E402

rng = np.random.default_rng(0)
x = rng.integers(0, 255, (4096, 28, 28, 1)).astype(np.uint8)
y = rng.integers(0, 10, 4096)
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
m.fit(x, y, batch_size=32, epochs=3, verbose=0)
torch.cuda.synchronize()
print("done")
