# %% [markdown]
# # Feature engineering: retail sales feature groups
# Mirrors notebooks/featurestore/hsfs/basics/feature_engineering.ipynb on the reference's own retail
# data: `stores data-set.csv` (45 stores) and `Features data set.csv` (8,190 exogenous rows) from
# notebooks/featurestore/hsfs/archive (bundled, `dataset.sample_data`).  The third file the notebook
# reads, `sales data-set.csv`, is stripped from the reference snapshot (.MISSING_LARGE_BLOBS), so
# weekly sales are synthetic over the real stores and dates.
# Steps: store_fg = stores joined with the distinct departments per store (:152-159, :177-182);
# weekly sales summed over the last 30/90/180/365 days per (store, dept) and per store — Spark's
# `F.sum("weekly_sales").over(Window.partitionBy(...).orderBy(timestamp).rangeBetween(days(-N), days(-1)))`
# (:222-249) as `featurestore.window` range sums (GPU window.hip kernel on large frames); sales_fg
# v1 / partitioned v2 / online v3 (:267-346); exogenous_fg with insert of the dates shifted by 365
# days, append_features, and a v2 that is deleted again (:367-484).
# %%
import numpy as np
import pandas as pd

import hsfs
from hops_examples_amd.dataset import sample_data
from hops_examples_amd.featurestore.window import days, with_range_sums

conn = hsfs.connection()
fs = conn.get_feature_store()
stores_csv = pd.read_csv(sample_data("retail/stores data-set.csv"))
exogenous_csv = pd.read_csv(sample_data("retail/Features data set.csv"))
assert stores_csv.shape == (45, 3) and exogenous_csv.shape == (8190, 12)

# synthetic weekly sales over the real stores and the exogenous file's weekly dates (2010-02-05 ..)
rng = np.random.default_rng(0)
weeks = pd.to_datetime(exogenous_csv.date[exogenous_csv.store == 1], format="%d/%m/%Y").iloc[:143]
store_ids = stores_csv.store.values[:6]
sales = pd.DataFrame([(s, d, day, rng.normal(20000, 4000)) for s in store_ids for d in range(1, 1 + (s % 3) + 2)
                      for day in weeks], columns=["store", "dept", "date", "weekly_sales"])

# %%
stores_depts_count = sales.groupby("store").dept.nunique().rename("num_depts").reset_index()
stores_fg = stores_csv.merge(stores_depts_count, on="store")  # inner join, as Spark's join
store_fg_meta = fs.create_feature_group(name="store_fg", version=1, primary_key=["store"],
                                        description="Store related features", time_travel_format=None,
                                        statistics_config={"enabled": True, "histograms": True,
                                                           "correlations": True})
store_fg_meta.save(stores_fg)

# %%
sales["timestamp"] = sales.date.astype("int64") // 10**9  # F.unix_timestamp("date")
periods = {"month": 30, "quarter": 90, "six_month": 180, "year": 365}
sales = with_range_sums(sales, {f"sales_last_{p}_store_dep": (days(-n), days(-1)) for p, n in periods.items()},
                        ["store", "dept"], "timestamp", "weekly_sales")
sales = with_range_sums(sales, {f"sales_last_{p}_store": (days(-n), days(-1)) for p, n in periods.items()},
                        "store", "timestamp", "weekly_sales")
sales = sales.drop(columns=["timestamp"]).fillna(0)
sales["date"] = sales.date.dt.strftime("%Y-%m-%d")

fg = fs.create_feature_group("sales_fg", version=1, description="Sales related features",
                             primary_key=["store", "dept", "date"], time_travel_format=None,
                             statistics_config={"enabled": True, "histograms": True, "correlations": True})
fg.save(sales.iloc[:-30])
fg.insert(sales.iloc[-30:])  # append the latest month
print(len(fg.read()), fg.get_statistics()["columns"][3]["mean"])
fs.create_feature_group("sales_fg", version=2, partition_key=["store"], description="Sales related features",
                        time_travel_format=None, statistics_config=False).save(sales)
fs.create_feature_group("sales_fg", version=3, primary_key=["store", "dept", "date"], online_enabled=True,
                        description="Sales related features", time_travel_format=None,
                        statistics_config=False).save(sales)

# %%
exogenous_fg = exogenous_csv.assign(date=pd.to_datetime(exogenous_csv.date, format="%d/%m/%Y").dt.strftime("%Y-%m-%d"))
exogenous_fg["is_holiday"] = exogenous_fg.is_holiday.astype(bool)
exo = fs.create_feature_group("exogenous_fg", version=1, primary_key=["store", "date"],
                              description="External features that influence sales, but are not under the control "
                                          "of the distribution chain", time_travel_format=None,
                              statistics_config={"enabled": True, "histograms": True, "correlations": True})
exo.save(exogenous_fg)
exogenous_fg_2013 = exogenous_fg.assign(
    date=(pd.to_datetime(exogenous_fg.date) + pd.Timedelta(days=365)).dt.strftime("%Y-%m-%d"))
fs.get_feature_group("exogenous_fg", 1).insert(exogenous_fg_2013)
exo = fs.get_feature_group("exogenous_fg", 1)
exo.append_features([hsfs.Feature("appended_feature", "double", default_value="10.0")])
exo.show(5)
v2 = fs.create_feature_group("exogenous_fg", version=2, primary_key=["store", "date"], time_travel_format=None,
                             statistics_config=False)
v2.save(exogenous_fg)
fs.get_feature_group("exogenous_fg", 2).delete()
print(len(exo.read()))
