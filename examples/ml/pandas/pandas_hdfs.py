# %% [markdown]
# # pandas CSV in the project (`hops.pandas_helper`), mirrors notebooks/ml/pandas/pandas-hdfs.ipynb
# %%
import pandas as pd

from hops import pandas_helper as pandas

df = pd.DataFrame({"a": [1, 2, 3], "b": ["x", "y", "z"]})
pandas.write_csv("Resources/df.csv", df)
print(pandas.read_csv("Resources/df.csv"))
