# %% [markdown]
# # LOCO ablation study on the Titanic training dataset (maggy)
# Mirrors notebooks/ml/Parallel_Experiments/Maggy/maggy-ablation-titanic-example.ipynb. The training dataset
# `titanic_train_dataset` v1 is created first (as notebooks/featurestore/datasets/TitanicTrainingDatasetPython
# does) from synthetic passengers.
# %%
import numpy as np
import pandas as pd

import hsfs
from maggy import experiment
from maggy.ablation import AblationStudy

rng = np.random.default_rng(0)
n = 891
df = pd.DataFrame({"pclass": rng.integers(1, 4, n), "sex": rng.integers(0, 2, n),
                   "fare": rng.gamma(2.0, 16.0, n).round(2), "age": rng.normal(30, 12, n).clip(1, 80).round(),
                   "sibsp": rng.integers(0, 5, n), "parch": rng.integers(0, 4, n)})
df["survived"] = ((df.sex == 1) ^ (rng.random(n) < 0.2)).astype(int)
fs = hsfs.connection().get_feature_store()
td = fs.create_training_dataset("titanic_train_dataset", version=1, data_format="tfrecord", label=["survived"])
td.save(df)

# %%
ablation_study = AblationStudy("titanic_train_dataset", training_dataset_version=1, label_name="survived")
ablation_study.features.include("pclass")
ablation_study.features.include(["fare", "sibsp"])
ablation_study.features.list_all()


def base_model_generator():
    from hops_examples_amd import keras as K

    model = K.Sequential()
    model.add(K.layers.Dense(64, activation="relu"))
    model.add(K.layers.Dense(64, name="my_dense_two", activation="relu"))
    model.add(K.layers.Dense(32, name="my_dense_three", activation="relu"))
    model.add(K.layers.Dense(32, name="my_dense_four", activation="relu"))
    model.add(K.layers.Dense(2, name="my_dense_sigmoid", activation="sigmoid"))
    model.add(K.layers.Dense(1, activation="linear"))
    return model


ablation_study.model.set_base_model_generator(base_model_generator)
ablation_study.model.layers.include("my_dense_two", "my_dense_three", "my_dense_four", "my_dense_sigmoid")
ablation_study.model.layers.include_groups(["my_dense_two", "my_dense_four"])
ablation_study.model.layers.include_groups(prefix="my_dense")
ablation_study.model.layers.print_all()
ablation_study.model.layers.print_all_groups()

# %%
def training_fn(dataset_function, model_function):
    from hops_examples_amd import keras as K

    model = model_function()
    model.compile(optimizer=K.optimizers.Adam(0.001), loss="binary_crossentropy", metrics=["accuracy"])
    history = model.fit(dataset_function(5, 10), epochs=5, steps_per_epoch=30, verbose=0)
    return float(history.history["accuracy"][-1])


result = experiment.lagom(train_fn=training_fn, experiment_type="ablation", ablation_study=ablation_study,
                          ablator="loco", name="Titanic-LOCO")
print(result)
