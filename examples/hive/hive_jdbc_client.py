# %% [markdown]
# # Hive over a JDBC connection with two-way TLS
# Mirrors hive/src/main/java/io/hops/examples/hive/HiveJDBCClient.java: read the credentials
# properties, connect to the HiveServer2 endpoint (`auth=noSasl;ssl=true;twoWay=true` with trust /
# key stores), create an external table over raw CSV data, copy it into an ORC table and query the
# average price per city.  The endpoint is a local `hive_server.HiveServer2` with throw-away
# certificates; synthetic Sacramento-style rows stand in for the raw data.
# %%
import numpy as np
import pandas as pd

from hops import hdfs
from hops_examples_amd import hive_server, tls

certs = tls.make_local_certs()
server = hive_server.HiveServer2(certfile=certs["server_cert"], keyfile=certs["server_key"], cafile=certs["ca"],
                                 two_way=True)
rng = np.random.default_rng(1)
n = 400
raw = pd.DataFrame({"street": [f"{i} OAK AVE" for i in range(n)], "city": rng.choice(["SACRAMENTO", "DAVIS", "GALT"], n),
                    "zip": rng.choice([95608, 95838], n), "state": "CA", "beds": rng.integers(1, 5, n),
                    "baths": rng.integers(1, 3, n), "sq__ft": rng.integers(500, 3000, n),
                    "type": rng.choice(["Residential", "Condo"], n), "sale_date": "Wed May 21 00:00:00 EDT 2008",
                    "price": rng.integers(50000, 500000, n), "latitude": rng.uniform(38.4, 38.7, n),
                    "longitude": rng.uniform(-121.5, -121.2, n)})
hdfs.mkdir("Resources/rawdata")
raw.to_csv(hdfs.project_path() + "Resources/rawdata/sales.csv", header=False, index=False)
with open("hive_credentials.properties", "w") as f:
    f.write(f"hive_url={server.url}\ndbname=default\ntruststore_path={certs['ca']}\ntruststore_pw=\n"
            f"keystore_path={certs['client_bundle']}\nkeystore_pw=\n")

# %%
props = hive_server.read_hive_credentials("hive_credentials.properties")
with hive_server.connect(hive_server.jdbc_url(props)) as conn:
    conn.createStatement().execute("set hive.exec.dynamic.partition.mode=nonstrict;")
    conn.createStatement().execute(
        "create external table sales(street string, city string, zip int, state string, beds int, baths int, "
        "sq__ft float, sales_type string, sale_date string, price float, latitude float, longitude float) "
        "ROW FORMAT DELIMITED FIELDS TERMINATED BY ',' LOCATION '/Projects/demo/Resources/rawdata'")
    conn.createStatement().execute(
        "create table orc_table (street string, city string, zip int, state string, beds int, baths int, "
        "sq__ft float, sales_type string, sale_date string, price float, latitude float, longitude float) "
        "STORED AS ORC")
    conn.createStatement().execute("insert overwrite table orc_table select * from sales")
    rst = conn.createStatement().executeQuery("select city, avg(price) as price from sales group by city")
    print("City \t Price")
    while rst.next():
        print(rst.getString(1) + "\t" + rst.getString(2))
server.close()
