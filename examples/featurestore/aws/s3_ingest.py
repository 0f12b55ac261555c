# %% [markdown]
# # S3 ingestion into the feature store, on the reference's own data
# Mirrors notebooks/featurestore/aws/s3/S3-Ingest-to-Feature-Store-basics.ipynb:100-110 (storage
# connector `telco_delta` -> CSV read from the bucket -> `telco_fg` keyed by customer_id with full
# statistics) and S3-Ingest-to-Feature-Store-housing-data.ipynb:74-90 (Sacramento housing CSV ->
# `housing_fg` keyed by latitude/longitude).  The bucket is a project directory holding the files the
# reference ships in notebooks/featurestore/aws/s3/data and aws/data (`dataset.sample_data`),
# including the `telco-delta` Delta table, which is read back through its transaction log too.
# %%
import hsfs
from hops import hdfs
from hops_examples_amd import dataset, delta
from hops_examples_amd.dataset import sample_data

fs = hsfs.connection().get_feature_store()
hdfs.mkdir("Resources/telco-bucket")
bucket = hdfs.project_path() + "Resources/telco-bucket"
dataset.upload(sample_data("telco/telco_customer_churn.csv"), "Resources/telco-bucket")
dataset.upload(sample_data("telco/telco-delta"), "Resources/telco-bucket")
dataset.upload(sample_data("Sacramentorealestatetransactions.csv"), "Resources/telco-bucket")

# %%
sc = fs.create_storage_connector("telco_delta", "S3", bucket=bucket)
sc = fs.get_storage_connector("telco_delta")
df = sc.read(data_format="csv", path=sc.bucket + "/telco_customer_churn.csv")
assert df.shape == (7043, 21), df.shape
telco_fg = fs.create_feature_group(name="telco_fg", version=1, description="On-demand FG with telecom data",
                                   primary_key=["customer_id"], time_travel_format=None,
                                   statistics_config={"enabled": True, "histograms": True, "correlations": True})
telco_fg.save(df)
stats = {c["column"]: c for c in telco_fg.get_statistics()["columns"]}
print(telco_fg.read().shape, "mean monthly_charges", round(stats["monthly_charges"]["mean"], 4))
assert abs(stats["monthly_charges"]["mean"] - df.monthly_charges.mean()) < 1e-6

# %% [markdown]
# The same rows as the bucket's Delta table (`_delta_log/00000000000000000000.json`: one WRITE commit, two
# snappy Parquet parts).
# %%
dl = delta.read(sc.bucket + "/telco-delta")
hist = delta.history(sc.bucket + "/telco-delta")
print(dl.shape, hist[["version", "operation"]].to_dict("records"))
assert dl.shape == (7043, 21) and list(hist.operation) == ["WRITE"]
assert set(dl.customer_id) == set(df.customer_id)

# %%
houses = sc.read(data_format="csv", path=sc.bucket + "/Sacramentorealestatetransactions.csv")
housing_fg = fs.create_feature_group(name="housing_fg", version=1, description="FG with Sacramento Housing Data",
                                     primary_key=["latitude", "longitude"], time_travel_format=None,
                                     statistics_config={"enabled": True, "histograms": True, "correlations": True})
housing_fg.save(houses)
print(housing_fg.read().shape)
