# %% [markdown]
# # Hive tables: external CSV -> partitioned ORC, SQL queries
# Mirrors notebooks/hive/PyHive.ipynb.  Uses a synthetic Sacramento-style file in RawData/.
# %%
import numpy as np
import pandas as pd

from hops import hdfs, hive

rng = np.random.default_rng(0)
n = 500
raw = pd.DataFrame({"street": [f"{i} MAIN ST" for i in range(n)], "city": rng.choice(["SACRAMENTO", "ELK GROVE"], n),
                    "zip": rng.choice([95608, 95838, 95823], n), "state": "CA", "beds": rng.integers(1, 5, n),
                    "baths": rng.integers(1, 3, n), "sq__ft": rng.integers(500, 3000, n),
                    "type": rng.choice(["Residential", "Condo"], n), "sale_date": "Wed May 21 00:00:00 EDT 2008",
                    "price": rng.integers(50000, 500000, n), "latitude": rng.uniform(38.4, 38.7, n),
                    "longitude": rng.uniform(-121.5, -121.2, n)})
hdfs.mkdir("RawData")
raw.to_csv(hdfs.project_path() + "RawData/sacramento.csv", header=False, index=False)
h = hive.setup_hive_connection()
h.execute("""CREATE EXTERNAL TABLE sacramento_properties_ext(street string, city string, zip int, state string,
beds int, baths int, sq__ft float, sales_type string, sale_date string, price float, latitude float, longitude float)
ROW FORMAT DELIMITED FIELDS TERMINATED BY ',' LOCATION '/Projects/demo/RawData'""")
print(h.execute("show tables"))

# %%
h.execute("""CREATE TABLE sacramento_properties(street string, city string, state string, beds int, baths int,
sq__ft float, sales_type string, sale_date string, price float, latitude float, longitude float)
PARTITIONED by (zip int) STORED AS ORC""")
h.execute("set hive.exec.dynamic.partition=true; set hive.exec.dynamic.partition.mode=nonstrict;")
h.execute("""INSERT OVERWRITE TABLE sacramento_properties PARTITION (zip)
SELECT street, city, state, beds, baths, sq__ft, sales_type, sale_date, price, latitude, longitude, zip
FROM sacramento_properties_ext""")
print(h.execute("select * FROM sacramento_properties WHERE zip=95608 LIMIT 10"))
print(h.execute("select sales_type, avg(price) as avg_price FROM sacramento_properties WHERE zip=95608 "
                "GROUP BY sales_type LIMIT 10"))
condos = h.cursor().execute("select * from sacramento_properties where `sales_type` = 'Condo'").fetchall()
print(len(condos))
