# %% [markdown]
# # SQL results to local plots (sparkmagic `%%sql -o` + matplotlib/seaborn stand-in)
# Mirrors notebooks/ml/Plotting/matplotlib_sparkmagic.ipynb:194-1309: query a Hive table from the
# "cluster" side, ship the result to the local pandas side (`%%sql -o df` / `%%local`), and plot
# distributions, group bars, a scatter and a correlation heat map.  The warehouse is the local
# Hive-style SQL engine; charts are SVG files in the project.  Synthetic Sacramento-style sales.
# %%
import numpy as np
import pandas as pd

from hops_examples_amd import hdfs, hive, notebook, plotting

rng = np.random.default_rng(0)
n = 985
cities = ["SACRAMENTO", "ELK GROVE", "ROSEVILLE", "CITRUS HEIGHTS", "ANTELOPE"]
sales = pd.DataFrame({"city": rng.choice(cities, n, p=[0.45, 0.2, 0.15, 0.1, 0.1]),
                      "beds": rng.integers(1, 6, n), "baths": rng.integers(1, 4, n),
                      "sq__ft": rng.integers(500, 4000, n)})
sales["price"] = (40000 + 95 * sales.sq__ft + 9000 * sales.beds + rng.normal(0, 30000, n)).round()
sales["latitude"] = rng.normal(38.58, 0.1, n)
sales["longitude"] = rng.normal(-121.4, 0.1, n)
hdfs.mkdir("RawData/sales")
sales.to_csv(hdfs.project_path() + "RawData/sales/sales.csv", header=False, index=False)
conn = hive.setup_hive_connection()
conn.execute(f"""CREATE EXTERNAL TABLE sacramento_sales(city string, beds int, baths int, sq__ft int, price float,
latitude float, longitude float) ROW FORMAT DELIMITED FIELDS TERMINATED BY ','
LOCATION '/Projects/{hdfs.project_name()}/RawData/sales'""")

# %%  %%sql -o prices  (the result lands in the local namespace as a pandas DataFrame)
ns = {}
notebook.sql("SELECT city, price, sq__ft, beds FROM sacramento_sales", output="prices", namespace=ns)
prices = ns["prices"]
by_city = notebook.sql("SELECT city, AVG(price) AS avg_price, COUNT(*) AS n FROM sacramento_sales GROUP BY city "
                       "ORDER BY avg_price DESC")

# %%  %%local: plot on the driver
plotting.save(plotting.histogram(prices.price, bins=30, title="price distribution", xlabel="USD"),
              "Resources/plots/price_hist.svg")
plotting.save(plotting.bar(by_city.city.tolist(), by_city.avg_price.to_numpy(), title="average price by city"),
              "Resources/plots/avg_price_by_city.svg")
plotting.save(plotting.scatter(prices.sq__ft, prices.price, title="price vs size", xlabel="sq ft", ylabel="USD"),
              "Resources/plots/price_vs_size.svg")
corr = prices[["price", "sq__ft", "beds"]].corr()
plotting.save(plotting.heatmap(corr.to_numpy(), labels=list(corr.columns), title="correlations"),
              "Resources/plots/corr.svg")
print(by_city)
assert abs(corr.loc["price", "sq__ft"]) > 0.8
