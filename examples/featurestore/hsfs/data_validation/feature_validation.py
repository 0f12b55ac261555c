# %% [markdown]
# # Data validation: rules -> expectations -> validation types
# Mirrors notebooks/featurestore/hsfs/data_validation/feature_validation_python.ipynb (rule catalogue,
# expectation with HAS_MIN/HAS_MAX, STRICT feature group rejecting bad inserts with the 417 message,
# WARNING/ALL/NONE, get_validations).
# %%
import pandas as pd

import hsfs
from hsfs.rule import Rule

conn = hsfs.connection()
fs = conn.get_feature_store()
print([r.to_dict()["name"] for r in conn.get_rules()][:5], "...")
expectation = fs.create_expectation("year", description="validate year correctness", features=["year"],
                                    rules=[Rule(name="HAS_MIN", level="ERROR", min=2018),
                                           Rule(name="HAS_MAX", level="WARNING", max=2021)])
expectation.save()

# %%
fg = fs.create_feature_group("economy_fg", 1, primary_key=["id"], time_travel_format="HUDI",
                             validation_type="STRICT", expectations=[expectation])
fg.save(pd.DataFrame({"id": [1, 2], "year": [2019, 2020], "salary": [1.0, 2.0]}))
try:
    fg.insert(pd.DataFrame({"id": [3], "year": [2022], "salary": [3.0]}))
except hsfs.ValidationError as e:
    print("rejected:", e)
fg.validation_type = "WARNING"
fg.insert(pd.DataFrame({"id": [3], "year": [2022], "salary": [3.0]}))
for v in fg.get_validations():
    print(v.to_dict()["validationTime"], v.status)
