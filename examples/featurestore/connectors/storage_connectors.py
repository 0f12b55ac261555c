# %% [markdown]
# # Storage connectors and on-demand feature groups
# Mirrors notebooks/featurestore/aws/s3 (bucket -> CSV -> feature group) and aws/redshift + hsfs/snowflake
# (on-demand feature groups over a SQL connector).  Local stand-ins: an S3-style connector is a directory,
# a JDBC-style connector is an SQLite database.
# %%
import sqlite3

import numpy as np
import pandas as pd

import hsfs
from hops import hdfs

fs = hsfs.connection().get_feature_store()
bucket = hdfs.project_path() + "Resources/bucket"
hdfs.mkdir("Resources/bucket")
rng = np.random.default_rng(0)
pd.DataFrame({"id": range(50), "median_income": rng.uniform(1, 10, 50), "house_value": rng.uniform(1e5, 5e5, 50)}) \
    .to_csv(bucket + "/housing.csv", index=False)
s3 = fs.create_storage_connector("housing_s3", "S3", bucket=bucket)
df = s3.read(data_format="csv", path=bucket + "/housing.csv")
fs.create_feature_group("housing_fg", 1, primary_key=["id"]).save(df)

# %%
db = hdfs.project_path() + "Resources/warehouse.db"
with sqlite3.connect(db) as c:
    pd.DataFrame({"customer_id": range(20), "churn_score": rng.random(20)}).to_sql("telco", c, index=False)
jdbc = fs.create_storage_connector("telco_redshift", "JDBC", connection_string=f"sqlite:///{db}")
od = fs.create_on_demand_feature_group("telco_on_dmd", version=1, storage_connector=jdbc,
                                       query="SELECT customer_id, churn_score FROM telco WHERE churn_score > 0.5")
od.save()
print(od.read().head())
