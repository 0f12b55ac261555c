# %% [markdown]
# # Train an MLP, export to the model registry, serve it (torch predictor, dynamic batching)
# Mirrors notebooks/ml/End_To_End_Pipeline/tensorflow/model_repo_and_serving.ipynb: flat 784 -> D128 relu ->
# D10 softmax (101,770 params), Adam 1e-3, export, get_best_model, create_or_update + start, REST inference.
# %%
import os

import numpy as np

from hops import model, serving
from hops_examples_amd import keras
from hops_examples_amd.models.zoo import mnist_mlp

FAST = os.environ.get("HOPSX_FAST") == "1"
rng = np.random.default_rng(0)
x = rng.random((640 if FAST else 6400, 784), dtype=np.float32)
y = (x[:, :10].argmax(1)).astype(np.int64)
m = mnist_mlp()
m.compile(keras.optimizers.Adam(1e-3), "sparse_categorical_crossentropy", ["accuracy"])
h = m.fit(x, y, batch_size=32, epochs=3, steps_per_epoch=None if FAST else 5, verbose=0)
acc = h.history["accuracy"][-1]

# %%
from hops_examples_amd.model import save_torch

save_torch(m.net, "mnist_mlp", builder="hops_examples_amd.models.zoo:mnist_mlp_net")
path = model.export("mnist_mlp", "mnist", metrics={"accuracy": acc})
print(model.get_best_model("mnist", "accuracy", model.Metric.MAX))

# %%
serving.create_or_update("mnist", path, model_version=1, model_server="TENSORFLOW_SERVING")
serving.start("mnist")
print(serving.make_inference_request("mnist", {"instances": x[:4].tolist()}))
serving.stop("mnist")
