# %% [markdown]
# # Delta tables: bulk insert, overwrite, time travel, MERGE upsert
# Mirrors notebooks/featurestore/delta/DeltaOnHops.ipynb (Scala/Spark there; pandas + Parquet here).
# %%
import pandas as pd

from hops import hdfs
from hops_examples_amd import delta

path = hdfs.project_path() + "Resources/hello_delta"
cols = ["id", "date", "value", "country"]
delta.write(pd.DataFrame([(1, "2019-02-30", 0.4151, "Sweden"), (2, "2019-05-01", 1.2151, "Ireland"),
                          (3, "2019-08-06", 0.2151, "Belgium"), (4, "2019-08-06", 0.8151, "Russia")], columns=cols), path)
delta.write(pd.DataFrame([(1, "2019-06-30", 0.4151, "Sweden"), (2, "2019-05-01", 1.2151, "Ireland"),
                          (3, "2017-08-06", 0.2151, "Belgium"), (4, "2019-08-06", 0.8151, "Russia")], columns=cols),
            path, mode="overwrite")
print(delta.read(path, version_as_of=0))
print(delta.read(path))

# %%
upsert = pd.DataFrame([(5, "2019-02-30", 0.7921, "Northern Ireland"), (1, "2019-05-01", 1.151, "Norway"),
                       (3, "2019-08-06", 0.999, "Belgium"), (6, "2019-08-06", 0.0151, "France")], columns=cols)
m = {c: f"newData.{c}" for c in cols}
(delta.DeltaTable.forPath(path).alias("oldData").merge(upsert, "oldData.id = newData.id")
 .whenMatched.update(m).whenNotMatched.insert(m).execute())
for v in range(3):
    print(f"version {v}:\n", delta.read(path, version_as_of=v))
print(delta.history(path))
