# %% [markdown]
# # Titanic training dataset preparation
# Mirrors notebooks/featurestore/datasets/TitanicTrainingDatasetPython.ipynb: fill missing age with 30,
# sex -> 0/1, cast to int, feature group with statistics, TFRecord TD `titanic_train_dataset` v1
# (consumed by the maggy ablation example).  Synthetic passengers (the raw CSV is not shipped).
# %%
import numpy as np
import pandas as pd

import hsfs

rng = np.random.default_rng(0)
n = 891
raw = pd.DataFrame({"pclass": rng.integers(1, 4, n), "sex": rng.choice(["male", "female"], n),
                    "age": np.where(rng.random(n) < 0.2, np.nan, rng.normal(30, 12, n).clip(1, 80)),
                    "sibsp": rng.integers(0, 5, n), "parch": rng.integers(0, 4, n), "fare": rng.gamma(2, 16, n)})
raw["survived"] = ((raw.sex == "female") ^ (rng.random(n) < 0.2)).astype(int)
clean = raw.assign(age=raw.age.fillna(30), sex=(raw.sex == "male").astype(int)).astype(
    {"age": int, "fare": float, "pclass": int})
fs = hsfs.connection().get_feature_store()
fg = fs.create_feature_group("titanic_training_all_features", 1, primary_key=["pclass", "sex", "age", "sibsp",
                                                                               "parch"],
                             statistics_config={"enabled": True, "histograms": True, "correlations": True})
fg.save(clean.drop_duplicates(["pclass", "sex", "age", "sibsp", "parch"]))
td = fs.create_training_dataset("titanic_train_dataset", version=1, data_format="tfrecord", label=["survived"])
td.save(fg.select_all())
print(td.read().head())
