# %% [markdown]
# # Training datasets: formats, splits, tf_data / torch_data
# Mirrors notebooks/featurestore/hsfs/basics/training_datasets.ipynb (TD from a query, csv/tfrecord/parquet,
# 0.7/0.2/0.1 splits with a seed, reading a split, tf_record_dataset(process=True) batches of ((32, 14), (32,))).
# %%
import numpy as np
import pandas as pd
import torch

import hsfs

fs = hsfs.connection().get_feature_store()
rng = np.random.default_rng(0)
n = 4000
cols = {f"f{i}": rng.normal(size=n) for i in range(13)}
df = pd.DataFrame({"id": np.arange(n), **cols, "weekly_sales": rng.normal(20000, 5000, n)})
fg = fs.create_feature_group("sales_features", 1, primary_key=["id"])
fg.save(df)

# %%
td = fs.create_training_dataset("sales_model", version=1, data_format="tfrecords",
                                splits={"train": 0.7, "test": 0.2, "validate": 0.1}, seed=42, label=["weekly_sales"])
td.save(fg.select_all())
print({s: len(td.read(s)) for s in ("train", "test", "validate")})

# %%
ds = td.tf_data(target_name="weekly_sales", split="train").tf_record_dataset(process=True, batch_size=32)
x, y = next(iter(ds))
print(x.shape, y.shape, x.dtype)

# %%
dev = "cuda" if torch.cuda.is_available() else "cpu"
loader = td.torch_data(target_name="weekly_sales", split="train", batch_size=256)
xb, yb = next(iter(loader))
print(xb.shape, xb.device, yb.shape)
