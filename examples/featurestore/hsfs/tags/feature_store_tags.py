# %% [markdown]
# # JSON-schema typed tags on feature groups and training datasets
# Mirrors notebooks/featurestore/hsfs/tags/feature_store_tags.ipynb.
# %%
import pandas as pd

import hsfs

fs = hsfs.connection().get_feature_store()
fs.create_tag_schema("data_owner", {"type": "object", "properties": {"owner": {"type": "string"},
                                                                    "team": {"type": "string"}},
                                    "required": ["owner"]})
fg = fs.create_feature_group("tagged_fg", 1, primary_key=["id"])
fg.save(pd.DataFrame({"id": [1, 2], "v": [0.1, 0.2]}))
fg.add_tag("data_owner", {"owner": "alice", "team": "ml"})
print(fg.get_tag("data_owner"), fg.get_tags())
try:
    fg.add_tag("data_owner", {"team": "no owner"})
except hsfs.FeatureStoreException as e:
    print("schema violation:", e)
fg.delete_tag("data_owner")
print(fg.get_tags())
