# %% [markdown]
# # Feature engineering: retail sales feature groups
# Mirrors notebooks/featurestore/hsfs/basics/feature_engineering.ipynb: weekly sales summed over the
# last 30/90/180/365 days per (store, dept) and per store — Spark's
# `F.sum("weekly_sales").over(Window.partitionBy(...).orderBy(timestamp).rangeBetween(days(-N), days(-1)))`
# (:229-249) as `featurestore.window` range sums (GPU window.hip kernel on large frames) — then feature
# groups with primary/partition keys, online flag and statistics, insert (append), append_features,
# delete.  Synthetic weekly retail data (the reference's sales CSV is not shipped).
# %%
import numpy as np
import pandas as pd

import hsfs
from hops_examples_amd.featurestore.window import days, with_range_sums

conn = hsfs.connection()
fs = conn.get_feature_store()
rng = np.random.default_rng(0)
weeks = pd.date_range("2010-02-05", periods=143, freq="7D")  # the retail data's weekly dates
sales = pd.DataFrame([(s, d, day, rng.normal(20000, 4000)) for s in range(1, 4) for d in range(1, 4) for day in weeks],
                     columns=["store", "dept", "date", "weekly_sales"])
sales["timestamp"] = sales.date.astype("int64") // 10**9  # F.unix_timestamp("date")
periods = {"month": 30, "quarter": 90, "six_month": 180, "year": 365}
sales = with_range_sums(sales, {f"sales_last_{p}_store_dep": (days(-n), days(-1)) for p, n in periods.items()},
                        ["store", "dept"], "timestamp", "weekly_sales")
sales = with_range_sums(sales, {f"sales_last_{p}_store": (days(-n), days(-1)) for p, n in periods.items()},
                        "store", "timestamp", "weekly_sales")
sales = sales.drop(columns=["timestamp"]).fillna(0)
sales["date"] = sales.date.dt.strftime("%Y-%m-%d")
days = weeks

# %%
fg = fs.create_feature_group("sales_fg", version=1, description="Sales related features",
                             primary_key=["store", "dept", "date"], partition_key=["store"], online_enabled=True,
                             statistics_config={"enabled": True, "histograms": True, "correlations": True})
fg.save(sales.iloc[:-30])
fg.insert(sales.iloc[-30:])  # append the latest month
print(len(fg.read()), fg.get_statistics()["columns"][3]["mean"])

# %%
fg.append_features([hsfs.Feature("holiday", "boolean", default_value=False)])
fg.show(5)
exo = fs.create_feature_group("exogenous_fg", version=1, primary_key=["store", "date"])
exo.save(pd.DataFrame({"store": np.repeat([1, 2, 3], len(days)), "date": np.tile(days.strftime("%Y-%m-%d"), 3),
                       "fuel_price": rng.uniform(2, 4, 3 * len(days)), "cpi": rng.uniform(200, 220, 3 * len(days))}))
tmp = fs.create_feature_group("scratch_fg", version=1, primary_key=["id"])
tmp.save(pd.DataFrame({"id": [1, 2], "v": [0.1, 0.2]}))
tmp.delete()
