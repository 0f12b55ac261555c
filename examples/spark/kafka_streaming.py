# %% [markdown]
# # Kafka -> streaming micro-batches -> CSV sink with checkpoint
# Mirrors notebooks/spark/KafkaSparkPython.ipynb (producer of N(0, 0.1) values, readStream from the topic,
# CSV sink with checkpointLocation, read back, histogram) and the Avro consumer of
# spark/.../StructuredStreamingKafka.scala (Parquet sink).
# %%
import numpy as np

from hops import kafka
from hops_examples_amd import avro, streaming

producer = kafka.Producer()
for v in np.random.default_rng(0).normal(0, 0.1, 200):
    producer.produce("numbers", value=str(v))
query = (streaming.read_stream("numbers")
         .select(lambda df: df.assign(x=df.value.astype(float))[["offset", "x"]])
         .write_stream(format="csv", path="Resources/numbers_csv", checkpoint_location="Resources/numbers_ckpt",
                       trigger_interval=0.1)
         .start())
query.process_all_available()
query.stop()
out = streaming.read_sink("Resources/numbers_csv")
print(len(out), np.histogram(out.x, bins=10)[0])

# %%
schema = {"type": "record", "name": "log", "fields": [{"name": "timestamp", "type": "string"},
                                                     {"name": "priority", "type": "string"},
                                                     {"name": "logger", "type": "string"},
                                                     {"name": "message", "type": "string"}]}
kafka.create_topic("logs", schema)
for i, p in enumerate(["INFO", "WARN", "INFO", "ERROR"]):
    producer.produce("logs", value=avro.encode(schema, {"timestamp": f"2020-01-0{i + 1}", "priority": p,
                                                        "logger": "app", "message": f"event {i}"}))
q = (streaming.read_stream("logs").from_avro()
     .write_stream(format="parquet", path="Resources/logs_parquet", checkpoint_location="Resources/logs_ckpt"))
q.process_all_available()
print(streaming.read_sink("Resources/logs_parquet", "parquet"))
