# %% [markdown]
# # Coalesced training dataset (single CSV file), mirrors
# notebooks/featurestore/hsfs/training/training-data-coalesced.ipynb
# %%
import numpy as np
import pandas as pd

import hsfs

fs = hsfs.connection().get_feature_store()
fg = fs.create_feature_group("coalesce_fg", 1, primary_key=["id"])
fg.save(pd.DataFrame({"id": np.arange(1000), "x": np.random.default_rng(0).normal(size=1000)}))
td = fs.create_training_dataset("coalesced_td", 1, data_format="csv", coalesce=True)
td.save(fg.select_all())
import glob, os
print(sorted(glob.glob(os.path.join(td.location, "**", "*.csv"), recursive=True)))
