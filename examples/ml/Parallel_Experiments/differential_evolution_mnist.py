# %% [markdown]
# # Differential evolution over kernel / pool / dropout (`experiment.differential_evolution`)
# Mirrors notebooks/ml/Parallel_Experiments/TensorFlow/evolutionary_search/evolutionary_search_mnist.ipynb
# (search_dict {'kernel': [2, 8], 'pool': [2, 8], 'dropout': [0.01, 0.99]}) and the PyTorch variant.
# %%
import os

from hops import experiment

FAST = os.environ.get("HOPSX_FAST") == "1"


def wrapper(kernel, pool, dropout):
    import numpy as np

    from hops_examples_amd import keras
    from hops_examples_amd.models.zoo import keras_mnist_cnn

    rng = np.random.default_rng(0)
    x = rng.integers(0, 128, (96 if FAST else 640, 28, 28, 1), dtype=np.uint8)
    y = rng.integers(0, 10, len(x))
    m = keras_mnist_cnn(kernel=kernel, pool=pool, dropout=dropout)
    m.compile(keras.optimizers.Adam(1e-3), "sparse_categorical_crossentropy", ["accuracy"])
    h = m.fit(x, y, batch_size=32, epochs=1, steps_per_epoch=None if FAST else 5, verbose=0)
    return {"metric": h.history["accuracy"][-1]}


# %%
search_dict = {"kernel": [2, 8], "pool": [2, 8], "dropout": [0.01, 0.99]}
best = experiment.differential_evolution(wrapper, search_dict, generations=1 if FAST else 4,
                                         population=4 if FAST else 5, direction="max", local_logdir=True)
print(best)
