# %% [markdown]
# # Grid search over learning rate x dropout (`experiment.grid_search`)
# Mirrors notebooks/ml/Parallel_Experiments/TensorFlow/grid_search/grid_search_fashion_mnist.ipynb:
# Conv32 k3 same -> Conv64 k3 same -> pool2 -> Dropout -> D128 -> Dropout -> D10 logits, Adam(lr),
# 6 trials run concurrently, one per GPU.
# %%
import os

from hops import experiment

FAST = os.environ.get("HOPSX_FAST") == "1"


def wrapper(learning_rate, dropout):
    import numpy as np

    from hops_examples_amd import keras
    from hops_examples_amd.models.zoo import fashion_mnist_cnn

    rng = np.random.default_rng(0)
    x = rng.integers(0, 128, (128 if FAST else 2048, 28, 28, 1), dtype=np.uint8)
    y = rng.integers(0, 10, len(x))
    for c in range(10):
        x[y == c, 2 * c:2 * c + 6, 4:10] += 120
    m = fashion_mnist_cnn(dropout=dropout)
    m.compile(keras.optimizers.Adam(learning_rate), "sparse_categorical_crossentropy", ["accuracy"])
    h = m.fit(x, y, batch_size=32, epochs=1 if FAST else 2, steps_per_epoch=None if FAST else 5, verbose=0)
    return {"accuracy": h.history["accuracy"][-1]}


# %%
args_dict = {"learning_rate": [0.001, 0.0005, 0.0001], "dropout": [0.45, 0.7]}
best_dir, best_params, best_metrics = experiment.grid_search(wrapper, args_dict, optimization_key="accuracy",
                                                             direction="max")
print(best_params, best_metrics)
