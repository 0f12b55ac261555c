# %% [markdown]
# # Time travel on HUDI feature groups
# Mirrors notebooks/featurestore/hsfs/time_travel/time_travel_python.ipynb (bulk insert via save, upserts via
# insert, commit_details, read(as of), read_changes between commits, Query.as_of across joined FGs).
# %%
import time

import pandas as pd

import hsfs

fs = hsfs.connection().get_feature_store()
fg = fs.create_feature_group("economy_fg", version=1, primary_key=["id"], partition_key=["year"],
                             hudi_precombine_key="id", time_travel_format="HUDI")
fg.save(pd.DataFrame({"id": [1, 2, 3, 4], "salary": [1000.0, 2000.0, 3000.0, 4000.0], "year": [2020] * 4}))
time.sleep(1.1)
fg.insert(pd.DataFrame({"id": [1, 2, 5], "salary": [1100.0, 2200.0, 5000.0], "year": [2020] * 3}))
details = fg.commit_details()
for k in sorted(details):
    print(k, details[k])
t0, t1 = [details[k]["committedOn"] for k in sorted(details)]

# %%
print(fg.read(t0))                      # the feature group as of the first commit
print(fg.read_changes(t0, t1))          # rows changed by the second commit
print(fg.select_all().as_of(t0).read())
