# %% [markdown]
# # Feature engineering: retail sales feature groups
# Mirrors notebooks/featurestore/hsfs/basics/feature_engineering.ipynb: rolling aggregates per store/dept
# over 30/90/180/365 days, feature groups with primary/partition keys, online flag and statistics,
# insert (append), append_features, delete.  Synthetic retail data (the reference CSV is not shipped).
# %%
import numpy as np
import pandas as pd

import hsfs

conn = hsfs.connection()
fs = conn.get_feature_store()
rng = np.random.default_rng(0)
days = pd.date_range("2021-01-01", periods=400, freq="D")
sales = pd.DataFrame([(s, d, day, rng.normal(20000, 4000)) for s in range(1, 4) for d in range(1, 4) for day in days],
                     columns=["store", "dept", "date", "weekly_sales"])
sales = sales.sort_values(["store", "dept", "date"])
for w in (30, 90, 180, 365):
    sales[f"sales_last_{w}_days"] = (sales.groupby(["store", "dept"]).weekly_sales
                                     .transform(lambda s: s.rolling(w, min_periods=1).mean()))
sales["date"] = sales.date.dt.strftime("%Y-%m-%d")

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
