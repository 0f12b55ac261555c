# %% [markdown]
# # Produce and consume project topics with Avro payloads
# Mirrors notebooks/kafka/KafkaPython.ipynb (producer/consumer config from hops.kafka + hops.tls, schema
# fetch, Avro decode).
# %%
from hops import kafka, tls
from hops_examples_amd import avro

schema = {"type": "record", "name": "test", "fields": [{"name": "name", "type": "string"},
                                                      {"name": "value", "type": "double"}]}
kafka.create_topic("test", schema)
config = {"bootstrap.servers": kafka.get_broker_endpoints(), "security.protocol": kafka.get_security_protocol(),
          "ssl.ca.location": tls.get_ca_chain_location(), "group.id": "demo"}
producer = kafka.Producer(config)
for i in range(10):
    producer.produce("test", value=avro.encode(schema, {"name": f"msg{i}", "value": i * 0.5}), key=str(i))
producer.flush()

# %%
consumer = kafka.Consumer({**config, "auto.offset.reset": "earliest"})
consumer.subscribe(["test"])
for _ in range(10):
    msg = consumer.poll(timeout=1.0)
    print(msg.key(), kafka.parse_avro_msg(msg, kafka.get_schema("test")))
consumer.close()
