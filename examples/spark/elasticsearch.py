# %% [markdown]
# # Write a DataFrame to an index and query it back
# Mirrors notebooks/spark/Elasticsearch-python.ipynb.
# %%
import pandas as pd

from hops import elasticsearch

config = elasticsearch.get_elasticsearch_config("newsgroup")
print(config)
df = pd.DataFrame({"id": [1, 2, 3], "text": ["gpu kernels", "hello world", "fast gpu"], "score": [1, 5, 9]})
elasticsearch.write(df, "newsgroup", id_field="id")
print(elasticsearch.read("newsgroup", {"query": {"match": {"text": "gpu"}}}))
print(elasticsearch.read("newsgroup", {"query": {"range": {"score": {"gte": 5}}}}))
