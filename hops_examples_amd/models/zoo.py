"""Keras-style builders for the small reference models (each returns an uncompiled
:class:`hops_examples_amd.keras.Sequential`; parameter counts match the reference).

| builder            | reference                                                              | params  |
|--------------------|------------------------------------------------------------------------|---------|
| simulated_mlp      | E4/E6 mirroredstrategy_simulated_data_example.ipynb:146-184 (D16-D1)    | 193     |
| titanic_dnn        | E13 maggy-ablation-titanic-example.ipynb:233-243                        | 7,813   |
| mnist_mlp          | E14 model_repo_and_serving.ipynb:202-223 (784-128-10)                   | 101,770 |
| maggy_regressor    | E12 maggy-pytorch-example.ipynb:46-100 (2-l1-l2-1, MSE)                 | varies  |
| keras_mnist_cnn    | E1 Experiment/Tensorflow/mnist.ipynb:154-164 (kernel/pool tunable, E11) | 239,594 |
| fashion_mnist_cnn  | E8/E9 grid_search_fashion_mnist.ipynb:149-258 (kernel/pool/dropout)     | 1,625,866 |
"""
from __future__ import annotations

from .. import keras as K


def simulated_mlp() -> K.Sequential:
    return K.Sequential([K.layers.Dense(16, activation="relu", input_shape=(10,)),
                         K.layers.Dense(1, activation="sigmoid")])


def titanic_dnn(n_features: int = 6) -> K.Sequential:
    return K.Sequential([
        K.layers.Dense(64, activation="relu", input_shape=(n_features,)),
        K.layers.Dense(64, name="my_dense_two", activation="relu"),
        K.layers.Dense(32, name="my_dense_three", activation="relu"),
        K.layers.Dense(32, name="my_dense_four", activation="relu"),
        K.layers.Dense(2, name="my_dense_sigmoid", activation="sigmoid"),
        K.layers.Dense(1, activation="linear"),
    ])


def mnist_mlp() -> K.Sequential:
    return K.Sequential([K.layers.Dense(128, activation="relu", input_shape=(784,)),
                         K.layers.Dense(10, activation="softmax")])


def maggy_regressor(l1_size: int = 8, l2_size: int = 8) -> K.Sequential:
    return K.Sequential([K.layers.Dense(l1_size, activation="relu", input_shape=(2,)),
                         K.layers.Dense(l2_size, activation="relu"),
                         K.layers.Dense(1)])


def keras_mnist_cnn(kernel: int = 4, pool: int = 4, dropout: float = 0.5) -> K.Sequential:
    return K.Sequential([
        K.layers.Conv2D(32, kernel_size=(kernel, kernel), activation="relu", input_shape=(28, 28, 1)),
        K.layers.Conv2D(64, (kernel, kernel), activation="relu"),
        K.layers.MaxPooling2D(pool_size=(pool, pool)),
        K.layers.Dropout(dropout),
        K.layers.Flatten(),
        K.layers.Dense(128, activation="relu"),
        K.layers.Dropout(dropout),
        K.layers.Dense(10, activation="softmax"),
    ])


def fashion_mnist_cnn(kernel: int = 3, pool: int = 2, dropout: float = 0.45) -> K.Sequential:
    return K.Sequential([
        K.layers.Conv2D(32, kernel_size=(kernel, kernel), padding="same", activation="relu", input_shape=(28, 28, 1)),
        K.layers.Conv2D(64, (kernel, kernel), padding="same", activation="relu"),
        K.layers.MaxPooling2D(pool_size=(pool, pool)),
        K.layers.Dropout(dropout),
        K.layers.Flatten(),
        K.layers.Dense(128, activation="relu"),
        K.layers.Dropout(dropout),
        K.layers.Dense(10),
    ])


def mnist_mlp_net():
    """The built module of :func:`mnist_mlp` (serving rebuilds exported models from this)."""
    m = mnist_mlp()
    m.build()
    return m.net
