"""Kafka-shaped topics, Avro payloads and checkpointed micro-batch streaming
(notebooks/kafka/KafkaPython.ipynb, notebooks/spark/KafkaSparkPython.ipynb,
spark/…/StructuredStreamingKafka.scala producer/consumer)."""
import numpy as np


def test_consumer_groups_and_offsets(project_root):
    from hops import kafka

    p = kafka.Producer(kafka.get_kafka_default_config())
    for i in range(5):
        p.produce("test", value=f"m{i}", key=str(i))
    p.flush()
    c = kafka.Consumer({"group.id": "g1", "auto.offset.reset": "earliest"})
    c.subscribe(["test"])
    got = [c.poll(1.0).value() for _ in range(3)]
    assert got == ["m0", "m1", "m2"]
    c2 = kafka.Consumer({"group.id": "g1"})  # same group resumes at the committed offset
    c2.subscribe(["test"])
    assert c2.poll(1.0).value() == "m3"
    late = kafka.Consumer({"group.id": "g2", "auto.offset.reset": "latest"})
    late.subscribe(["test"])
    assert late.poll(0.05) is None
    p.produce("test", value=b"\x00\x01binary")
    assert late.poll(1.0).value() == b"\x00\x01binary"


def test_avro_kafka_roundtrip(project_root):
    from hops import kafka
    from hops_examples_amd import avro

    schema = {"type": "record", "name": "log", "fields": [
        {"name": "timestamp", "type": "string"}, {"name": "priority", "type": "string"},
        {"name": "logger", "type": "string"}, {"name": "message", "type": ["null", "string"]}]}
    kafka.create_topic("logs", schema)
    rows = [{"timestamp": "2020-01-01", "priority": "INFO", "logger": "a", "message": "hello"},
            {"timestamp": "2020-01-02", "priority": "WARN", "logger": "b", "message": None}]
    p = kafka.Producer()
    for r in rows:
        p.produce("logs", value=avro.encode(schema, r))
    c = kafka.Consumer({"group.id": "x"})
    c.subscribe(["logs"])
    dec = [kafka.parse_avro_msg(c.poll(1.0), kafka.get_schema("logs")) for _ in rows]
    assert dec == rows


def test_stream_to_csv_exactly_once(project_root):
    from hops import kafka
    from hops_examples_amd import streaming

    p = kafka.Producer()
    vals = np.random.default_rng(0).normal(0, 0.1, 20)
    for v in vals[:12]:
        p.produce("numbers", value=str(v))
    q = (streaming.read_stream("numbers")
         .select(lambda df: df.assign(x=df.value.astype(float))[["offset", "x"]])
         .write_stream(format="csv", path="Resources/stream_out", checkpoint_location="Resources/ckpt",
                       trigger_interval=0.05).start())
    q.process_all_available()
    q.stop()
    for v in vals[12:]:
        p.produce("numbers", value=str(v))
    # a new query on the same checkpoint resumes where the first stopped: no duplicates, no gaps
    q2 = (streaming.read_stream("numbers")
          .select(lambda df: df.assign(x=df.value.astype(float))[["offset", "x"]])
          .write_stream(format="csv", path="Resources/stream_out", checkpoint_location="Resources/ckpt"))
    q2.process_all_available()
    out = streaming.read_sink("Resources/stream_out", "csv")
    assert out.offset.tolist() == list(range(20))
    np.testing.assert_allclose(out.x.to_numpy(), vals)
