# %% [markdown]
# # Feature exploration: select / filter / join / SQL
# Mirrors notebooks/featurestore/hsfs/basics/feature_exploration.ipynb (get_feature_group with the default
# version warning, show, select, filter with & and |, implicit-key joins, to_string, fs.sql).
# %%
import numpy as np
import pandas as pd

import hsfs

fs = hsfs.connection().get_feature_store()
rng = np.random.default_rng(0)
sales = pd.DataFrame({"store": rng.integers(1, 5, 300), "dept": rng.integers(1, 9, 300), "date": rng.integers(0, 30, 300),
                      "weekly_sales": rng.normal(20000, 5000, 300)}).drop_duplicates(["store", "dept", "date"])
fs.create_feature_group("sales_fg", 1, primary_key=["store", "dept", "date"]).save(sales)
exo = pd.DataFrame([(s, d, rng.uniform(2, 4), rng.uniform(200, 220)) for s in range(1, 5) for d in range(30)],
                   columns=["store", "date", "fuel_price", "cpi"])
fs.create_feature_group("exogenous_fg", 1, primary_key=["store", "date"]).save(exo)

# %%
sales_fg = fs.get_feature_group("sales_fg")  # VersionWarning: defaulting to version 1
exogenous_fg = fs.get_feature_group("exogenous_fg", version=1)
sales_fg.show(5)
q = sales_fg.select(["store", "dept", "weekly_sales"]).join(exogenous_fg.select(["fuel_price"]))
print(q.to_string())
q.show(5)

# %%
q2 = (sales_fg.select_all()
      .join(exogenous_fg.select(["fuel_price", "cpi"]).filter((exogenous_fg.fuel_price <= 2.7) | (exogenous_fg.cpi > 215)))
      .filter((sales_fg.weekly_sales >= 20000) & (sales_fg.dept != 3)))
print(q2.to_string())
print(len(q2.read()))
print(fs.sql("SELECT store, AVG(weekly_sales) AS avg_sales FROM sales_fg_1 GROUP BY store"))
