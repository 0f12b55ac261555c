# %% [markdown]
# # MNIST CNN with `experiment.launch` (Keras-style API on MI355X kernels)
# Mirrors notebooks/ml/Experiment/Tensorflow/mnist.ipynb: Conv32 k4 -> Conv64 k4 -> MaxPool4 ->
# Dropout .5 -> Dense128 -> Dropout .5 -> Dense10 softmax, Adadelta(1.0), batch 32,
# TensorBoard logdir, model export to the registry. Synthetic MNIST-shaped data.
# %%
import os

from hops import experiment, model as hopsworks_model, tensorboard

FAST = os.environ.get("HOPSX_FAST") == "1"


def keras_mnist():
    import numpy as np

    from hops_examples_amd import keras
    from hops_examples_amd.models.zoo import keras_mnist_cnn

    rng = np.random.default_rng(0)
    x = rng.integers(0, 128, (320 if FAST else 6400, 28, 28, 1), dtype=np.uint8)
    y = rng.integers(0, 10, len(x))
    for c in range(10):  # a learnable synthetic task: a bright block whose position encodes the class
        x[y == c, 2 * c:2 * c + 6, 4:10] += 120
    m = keras_mnist_cnn()
    m.compile(optimizer=keras.optimizers.Adadelta(1.0), loss="sparse_categorical_crossentropy",
              metrics=["accuracy"])
    tb = keras.callbacks.TensorBoard(log_dir=tensorboard.logdir())
    h = m.fit(x, y, batch_size=32, epochs=1 if FAST else 10, steps_per_epoch=None if FAST else 10,
              callbacks=[tb], verbose=1)
    loss, acc = m.evaluate(x[:320], y[:320], batch_size=10, verbose=0)
    m.save("mnist_cnn.pt")
    hopsworks_model.export("mnist_cnn.pt", "mnist", metrics={"accuracy": acc})
    return {"accuracy": acc, "loss": loss}


# %%
logdir, result = experiment.launch(keras_mnist, name="keras mnist", local_logdir=True, metric_key="accuracy")
print(logdir, result)
