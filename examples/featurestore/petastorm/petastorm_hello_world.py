# %% [markdown]
# # Petastorm datasets: Unischema, codecs, readers, sharding, torch DataLoader
# Mirrors notebooks/featurestore/petastorm/PetastormHelloWorld.ipynb.
# %%
import numpy as np
import pandas as pd

from hops import featurestore, hdfs
from petastorm import make_batch_reader, make_reader
from petastorm.codecs import CompressedImageCodec, NdarrayCodec, ScalarCodec
from petastorm.etl.dataset_metadata import materialize_dataset, write_rows
from petastorm.predicates import in_lambda
from petastorm.pytorch import DataLoader
from petastorm.types import IntegerType
from petastorm.unischema import Unischema, UnischemaField

HelloWorldSchema = Unischema("HelloWorldSchema", [
    UnischemaField("id", np.int32, (), ScalarCodec(IntegerType()), False),
    UnischemaField("image1", np.uint8, (128, 256, 3), CompressedImageCodec("png"), False),
    UnischemaField("array_4d", np.uint8, (None, 128, 30, None), NdarrayCodec(), False),
])
print(HelloWorldSchema.as_spark_schema())
OUTPUT_URL = hdfs.project_path() + "Resources/hello_world"


def row_generator(x):
    return {"id": x, "image1": np.random.randint(0, 255, dtype=np.uint8, size=(128, 256, 3)),
            "array_4d": np.random.randint(0, 255, dtype=np.uint8, size=(4, 128, 30, 3))}


with materialize_dataset(None, OUTPUT_URL, HelloWorldSchema, 256):
    write_rows(OUTPUT_URL, HelloWorldSchema, [row_generator(i) for i in range(10)], rows_per_group=2)

# %%
with make_reader(OUTPUT_URL) as reader:
    for sample in reader:
        print(sample.id)
with DataLoader(make_reader(OUTPUT_URL), batch_size=4) as train_loader:
    print(next(iter(train_loader))["id"])
with make_reader(OUTPUT_URL, schema_fields=["array_4d", "id"], shard_count=2, cur_shard=1) as reader:
    print([s.id for s in reader])
with make_reader(OUTPUT_URL, predicate=in_lambda(["id"], lambda id: id == 5)) as reader:
    print([s.id for s in reader])

# %%
import pyarrow as pa
import pyarrow.parquet as pq

OUTPUT_URL2 = hdfs.project_path() + "Resources/hello_world_external"
hdfs._resolve(OUTPUT_URL2).mkdir(parents=True, exist_ok=True)
pq.write_table(pa.Table.from_pandas(pd.DataFrame({"id": range(10), "value1": np.random.randint(-255, 255, 10),
                                                  "value2": np.random.randint(-255, 255, 10)})),
               str(hdfs._resolve(OUTPUT_URL2) / "part-0.parquet"))
with make_batch_reader(OUTPUT_URL2, schema_fields=["id", "value1", "value2"]) as reader:
    for schema_view in reader:
        print("Batched read:\nid: {0} value1: {1} value2: {2}".format(schema_view.id, schema_view.value1,
                                                                      schema_view.value2))

# %%
TestSchema = Unischema("TestSchema", [UnischemaField(c, np.int32, (), ScalarCodec(IntegerType()), False)
                                      for c in "ABCD"])
pandas_df = pd.DataFrame(np.random.randint(0, 100, size=(100, 4)), columns=list("ABCD"))
featurestore.create_training_dataset(pandas_df, "petastorm_hello_world", data_format="petastorm",
                                     petastorm_args={"schema": TestSchema})
print(featurestore.get_training_dataset("petastorm_hello_world").head())
