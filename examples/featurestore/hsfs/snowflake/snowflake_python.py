# %% [markdown]
# # Snowflake: Python connector, Spark connector and on-demand feature groups
# Mirrors notebooks/featurestore/hsfs/snowflake/python.ipynb:51-488 and getting-started.ipynb:113-150
# (`connector.snowflake_connector_options()` -> `snowflake.connector.connect` -> query CUSTOMER_CHURN into
# pandas), pyspark.ipynb:92-192 (`spark_options()` + "query" -> `spark.read.format("net.snowflake.spark.snowflake")`,
# an on-demand feature group with statistics, `select(...).show(5)`) and scala.ipynb:84-207 (the same
# on-demand group through the builder API).  The warehouse is the local stand-in (hops_examples_amd.snowflake),
# seeded with the reference's telco churn CSV; the password comes from the environment, as it should.
# %%
import os

import pandas as pd

import hsfs
import snowflake.connector
from hops_examples_amd.dataset import sample_data
from hops_examples_amd.livy import SparkStandIn
from snowflake.connector import write_pandas

os.environ.setdefault("SNOWFLAKE_PASSWORD", "local-only")
spark = SparkStandIn()
connection = hsfs.connection()
fs = connection.get_feature_store()
fs.create_storage_connector("sfconnector", "SNOWFLAKE",
                            options={"url": "https://hopsx.snowflakecomputing.com", "user": "analyst",
                                     "database": "TELCO_DB", "schema": "PUBLIC", "warehouse": "COMPUTE_WH",
                                     "role": "ANALYST"})

# seed the warehouse: the reference's telco data as CUSTOMER_CHURN and TELCO (upper-case identifiers)
telco_csv = pd.read_csv(sample_data("telco/telco_customer_churn.csv"))
connector = fs.get_storage_connector("sfconnector")
with snowflake.connector.connect(**connector.snowflake_connector_options()) as seed:
    write_pandas(seed, telco_csv, "CUSTOMER_CHURN", overwrite=True)
    write_pandas(seed, telco_csv, "TELCO", overwrite=True)

# %% [markdown]
# ## Python connector (python.ipynb / getting-started.ipynb)
# %%
sfConnectorOptions = connector.snowflake_connector_options()
assert "password" in sfConnectorOptions and sfConnectorOptions["account"] == "hopsx"
ctx = snowflake.connector.connect(**sfConnectorOptions)
cs = ctx.cursor()
allrows = cs.execute("""select CUSTOMER_ID,GENDER,SENIOR_CITIZEN,PARTNER,DEPENDENTS,TENURE,PHONE_SERVICE,
                             MULTIPLE_LINES,INTERNET_SERVICE,ONLINE_SECURITY,ONLINE_BACKUP,DEVICE_PROTECTION,
                             TECH_SUPPORT,STREAMING_TV,STREAMING_MOVIES,CONTRACT,PAPERLESS_BILLING,
                             PAYMENT_METHOD,MONTHLY_CHARGES,TOTAL_CHARGES,CHURN from CUSTOMER_CHURN """).fetchall()
churn = pd.DataFrame(allrows)
churn.columns = ['Customer_Id', 'Gender', 'Senior_Citizen', 'Partner', 'Dependents', 'Tenure', 'Phone_Service',
                 'Multiple_Lines', 'Internet_Service', 'Online_Security', 'Online_Backup', 'Device_Protection',
                 'Tech_Support', 'Streaming_Tv', 'Streaming_Movies', 'Contract', 'Paperless_Billing',
                 'Payment_Method', 'Monthly_Charges', 'Total_Charges', 'Churn?']
print(churn.shape)
assert churn.shape == (7043, 21)
print(churn.groupby("Contract")["Churn?"].apply(lambda s: (s == "Yes").mean()).round(3).to_dict())
ctx.close()

# %% [markdown]
# ## Spark connector and an on-demand feature group (pyspark.ipynb)
# %%
snowflake_conn = fs.get_storage_connector("sfconnector")
sfOptions = snowflake_conn.spark_options()
sfOptions["query"] = "select * from TELCO"
df = spark.read.format("net.snowflake.spark.snowflake").options(**sfOptions).load()
df.show(10)
telco_on_dmd = fs.create_on_demand_feature_group(name="telco_snowflake", version=2, query="select * from telco",
                                                 description="On-demand feature group for telecom customer data",
                                                 storage_connector=snowflake_conn, statistics_config=True)
telco_on_dmd.save()
telco_on_dmd.select(['customer_id', 'internet_service', 'phone_service', 'total_charges', 'churn']).show(5)
assert telco_on_dmd.read().shape == (7043, 21)

# %% [markdown]
# ## The same through the builder API (scala.ipynb)
# %%
telcoOnDmd = (fs.createOnDemandFeatureGroup()
              .name("telco_snowflake_scala").version(1).query("select * from CUSTOMER_CHURN")
              .description("On-demand feature group for telecom customer data")
              .storageConnector(snowflake_conn).statisticsConfig(hsfs.StatisticsConfig(True, True, True))
              .build())
telcoOnDmd.save()
telcoOnDmd.select(["customer_id", "internet_service", "phone_service", "total_charges", "churn"]).show(5)
