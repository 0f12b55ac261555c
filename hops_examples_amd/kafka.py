"""Project message topics (``hops.kafka`` / ``hops.tls`` surface) backed by
append-only JSON-lines logs under ``Logs/Kafka/<topic>.jsonl``.

The reference streams inference logs to a Kafka topic ``<serving>-inf<id>`` and
consumes them with ``confluent_kafka`` + Avro (IrisClassification_And_Serving_SKLearn.ipynb:905-1031,
notebooks/kafka/KafkaPython.ipynb).  A hosted broker is platform
infrastructure, so topics here are local logs with the same producer /
consumer shape (``produce``/``flush``, ``subscribe``/``poll``) and the same
record schema; an Avro-style schema registry is kept per topic.
"""
from __future__ import annotations

import json
import threading
import time
from pathlib import Path

from . import hdfs

_lock = threading.Lock()

INFERENCE_SCHEMA = {
    "type": "record",
    "name": "inferencelog",
    "fields": [
        {"name": "modelId", "type": "int"},
        {"name": "modelName", "type": "string"},
        {"name": "modelVersion", "type": "int"},
        {"name": "requestTimestamp", "type": "long"},
        {"name": "responseHttpCode", "type": "int"},
        {"name": "inferenceRequest", "type": "string"},
        {"name": "inferenceResponse", "type": "string"},
        {"name": "modelServer", "type": "string"},
        {"name": "servingTool", "type": "string"},
    ],
}


def _dir() -> Path:
    d = Path(hdfs.project_path()) / "Logs" / "Kafka"
    d.mkdir(parents=True, exist_ok=True)
    return d


def topic_path(topic: str) -> Path:
    return _dir() / f"{topic}.jsonl"


def create_topic(topic: str, schema: dict | None = None) -> None:
    topic_path(topic).touch()
    if schema is not None:
        (_dir() / f"{topic}.schema.json").write_text(json.dumps(schema))


def get_schema(topic: str) -> str:
    p = _dir() / f"{topic}.schema.json"
    return p.read_text() if p.exists() else json.dumps(INFERENCE_SCHEMA)


def get_broker_endpoints() -> str:
    return "file://" + str(_dir())


def get_security_protocol() -> str:
    return "PLAINTEXT"


def get_kafka_default_config() -> dict:
    return {"bootstrap.servers": get_broker_endpoints(), "security.protocol": get_security_protocol(),
            "group.id": "hopsx", "auto.offset.reset": "earliest"}


def append(topic: str, value, key=None) -> None:
    rec = {"timestamp": time.time(), "key": key, "value": value}
    with _lock:
        with open(topic_path(topic), "a") as f:
            f.write(json.dumps(rec, default=str) + "\n")


class Message:
    def __init__(self, topic, rec, offset):
        self._topic, self._rec, self._offset = topic, rec, offset

    def value(self):
        v = self._rec["value"]
        return v if isinstance(v, (bytes, str)) else json.dumps(v)

    def key(self):
        return self._rec.get("key")

    def topic(self):
        return self._topic

    def offset(self):
        return self._offset

    def timestamp(self):
        return (0, int(self._rec["timestamp"] * 1000))

    def error(self):
        return None


class Producer:
    def __init__(self, config: dict | None = None):
        self.config = config or {}

    def produce(self, topic, value=None, key=None, callback=None, **kw):
        append(topic, value.decode() if isinstance(value, bytes) else value, key)
        if callback:
            callback(None, None)

    def poll(self, timeout=0):
        return 0

    def flush(self, timeout=None):
        return 0


class Consumer:
    def __init__(self, config: dict | None = None):
        self.config = config or {}
        self._topics: list[str] = []
        self._offsets: dict[str, int] = {}

    def subscribe(self, topics):
        self._topics = list(topics)
        for t in self._topics:
            self._offsets.setdefault(t, 0)

    def poll(self, timeout: float = 1.0):
        deadline = time.time() + (timeout or 0)
        while True:
            for t in self._topics:
                p = topic_path(t)
                if not p.exists():
                    continue
                lines = p.read_text().splitlines()
                off = self._offsets[t]
                if off < len(lines):
                    self._offsets[t] = off + 1
                    return Message(t, json.loads(lines[off]), off)
            if time.time() >= deadline:
                return None
            time.sleep(0.01)

    def close(self):
        pass


def parse_avro_msg(msg, avro_schema=None) -> dict:
    """Messages are JSON-encoded records of the topic schema."""
    v = msg if isinstance(msg, (bytes, str)) else msg.value()
    if isinstance(v, bytes):
        v = v.decode()
    return json.loads(v) if isinstance(v, str) else v


def convert_json_schema_to_avro(schema):
    return schema if isinstance(schema, dict) else json.loads(schema)


# ---- hops.tls surface: certificate locations of the project (local placeholders)
def get_ca_chain_location() -> str:
    return str(_dir() / "ca_chain.pem")


def get_client_certificate_location() -> str:
    return str(_dir() / "client.pem")


def get_client_key_location() -> str:
    return str(_dir() / "client_key.pem")
