# %% [markdown]
# # On-demand feature group over a SQL warehouse -> indexed features -> online HUDI feature group
# Mirrors notebooks/featurestore/aws/redshift/Redshift_pyspark.ipynb:129-305: an on-demand feature
# group defined by a SQL query over a Redshift storage connector, read back as a dataframe,
# categorical columns indexed (Spark `StringIndexer`: labels ordered by frequency, indices as
# doubles), then saved as an online-enabled HUDI feature group keyed by customerID.  The warehouse
# is a local SQLite database behind a JDBC-style connector (no cluster); the telco churn rows are
# synthetic with the dataset's column names.
# %%
import sqlite3

import numpy as np
import pandas as pd

import hsfs
from hops import hdfs

rng = np.random.default_rng(0)
n = 500
telco = pd.DataFrame({
    "customerID": [f"{i:04d}-CUST" for i in range(n)], "gender": rng.choice(["Male", "Female"], n),
    "SeniorCitizen": rng.integers(0, 2, n), "Partner": rng.choice(["Yes", "No"], n),
    "Dependents": rng.choice(["Yes", "No"], n, p=[0.3, 0.7]), "tenure": rng.integers(0, 72, n),
    "PhoneService": rng.choice(["Yes", "No"], n, p=[0.9, 0.1]),
    "Contract": rng.choice(["Month-to-month", "One year", "Two year"], n, p=[0.55, 0.25, 0.2]),
    "PaymentMethod": rng.choice(["Electronic check", "Mailed check", "Bank transfer", "Credit card"], n),
    "MonthlyCharges": rng.uniform(18, 120, n).round(2), "Churn": rng.choice(["Yes", "No"], n, p=[0.27, 0.73])})
db = hdfs.project_path() + "Resources/redshift_warehouse.db"
hdfs.mkdir("Resources")
with sqlite3.connect(db) as c:
    telco.to_sql("telco", c, index=False, if_exists="replace")

# %%
fs = hsfs.connection().get_feature_store()
connector = fs.create_storage_connector("telco_redshift_cluster", "REDSHIFT", connection_string=f"jdbc:sqlite:{db}",
                                        options={"table": "telco"})
telco_on_dmd = fs.create_on_demand_feature_group(name="telco_redshift", version=1, query="select * from telco",
                                                 description="On-demand feature group for telecom customer data",
                                                 storage_connector=connector, statistics_config=False)
telco_on_dmd.save()
telco_df = telco_on_dmd.read()
telco_on_dmd.show(5)


# %%
def string_indexer(col: pd.Series) -> pd.Series:
    """Spark ML StringIndexer: the most frequent label gets 0.0 (ties by label), output is double."""
    vc = col.value_counts()
    order = sorted(vc.index, key=lambda v: (-vc[v], v))
    return col.map({v: float(i) for i, v in enumerate(order)})


categorical = ["gender", "Partner", "Dependents", "PhoneService", "Contract", "PaymentMethod", "Churn"]
indexed = telco_df.copy()
for c in categorical:
    indexed[c + "_index"] = string_indexer(indexed[c])
indexed = indexed.drop(columns=categorical)
assert indexed["Contract_index"].eq(0.0).sum() == telco_df["Contract"].value_counts().max()

# %%
telco_fg = fs.create_feature_group(name="telco_customer_features", version=1, primary_key=["customerID"],
                                   description="Telecom customer features", time_travel_format="HUDI",
                                   online_enabled=True,
                                   statistics_config={"enabled": True, "histograms": True, "correlations": True})
telco_fg.save(indexed)
print(telco_fg.read().head())
td = fs.create_training_dataset("telco_churn_td", version=1, data_format="csv", label=["Churn_index"])
td.save(telco_fg.select_all())
td.init_prepared_statement()
print(td.get_serving_vector({"customerID": "0007-CUST"}))
