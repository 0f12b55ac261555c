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

import base64
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


def append(topic: str, value, key=None) -> int:
    """Append one record; bytes payloads (e.g. Avro) are stored base64-encoded. Returns its offset."""
    rec = {"timestamp": time.time(), "key": key.decode() if isinstance(key, bytes) else key}
    if isinstance(value, (bytes, bytearray)):
        rec["value_b64"] = base64.b64encode(bytes(value)).decode()
    else:
        rec["value"] = value
    with _lock:
        p = topic_path(topic)
        with open(p, "a") as f:
            f.write(json.dumps(rec, default=str) + "\n")
        _counts[topic] = _counts.get(topic, _count_lines(p) - 1) + 1
        return _counts[topic] - 1


_counts: dict = {}


def _count_lines(p: Path) -> int:
    if not p.exists():
        return 0
    with open(p, "rb") as f:
        return sum(1 for _ in f)


def end_offset(topic: str) -> int:
    return _count_lines(topic_path(topic))


class Message:
    def __init__(self, topic, rec, offset):
        self._topic, self._rec, self._offset = topic, rec, offset

    def value(self):
        if "value_b64" in self._rec:
            return base64.b64decode(self._rec["value_b64"])
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

    def produce(self, topic, value=None, key=None, callback=None, on_delivery=None, **kw):
        off = append(topic, value, key)
        cb = callback or on_delivery
        if cb:
            cb(None, Message(topic, {"timestamp": time.time(), "key": key, "value": None}, off))

    def poll(self, timeout=0):
        return 0

    def flush(self, timeout=None):
        return 0


class Consumer:
    """Per-topic byte cursors (no re-reading), committed offsets per ``group.id``
    (``Logs/Kafka/<topic>.offsets.<group>``), ``auto.offset.reset`` earliest|latest."""

    def __init__(self, config: dict | None = None):
        self.config = config or {}
        self.group = str(self.config.get("group.id", "hopsx"))
        self.auto_commit = str(self.config.get("enable.auto.commit", "true")).lower() == "true"
        self._topics: list[str] = []
        self._pos: dict[str, tuple[int, int]] = {}  # topic -> (record offset, byte position)

    def _committed(self, t):
        p = _dir() / f"{t}.offsets.{self.group}"
        return int(p.read_text()) if p.exists() else None

    def _seek(self, t, off):
        p = topic_path(t)
        pos, n = 0, 0
        if p.exists():
            with open(p, "rb") as f:
                while n < off:
                    line = f.readline()
                    if not line:
                        break
                    pos += len(line)
                    n += 1
        self._pos[t] = (n, pos)

    def subscribe(self, topics):
        self._topics = list(topics)
        for t in self._topics:
            c = self._committed(t)
            if c is None:
                c = 0 if self.config.get("auto.offset.reset", "earliest") in ("earliest", "smallest") else \
                    end_offset(t)
            self._seek(t, c)

    def assign_offset(self, topic, offset):
        self._seek(topic, offset)

    def poll(self, timeout: float = 1.0):
        deadline = time.time() + (timeout or 0)
        while True:
            for t in self._topics:
                p = topic_path(t)
                if not p.exists():
                    continue
                off, pos = self._pos[t]
                with open(p, "rb") as f:
                    f.seek(pos)
                    line = f.readline()
                if line.endswith(b"\n"):
                    self._pos[t] = (off + 1, pos + len(line))
                    if self.auto_commit:
                        self.commit(topic=t)
                    return Message(t, json.loads(line), off)
            if time.time() >= deadline:
                return None
            time.sleep(0.005)

    def consume(self, num_messages: int = 1, timeout: float = 1.0) -> list:
        out = []
        for _ in range(num_messages):
            m = self.poll(timeout if not out else 0)
            if m is None:
                break
            out.append(m)
        return out

    def commit(self, message=None, topic=None, asynchronous: bool = False):
        for t in ([topic] if topic else self._topics):
            (_dir() / f"{t}.offsets.{self.group}").write_text(str(self._pos[t][0]))

    def position(self, topic):
        return self._pos[topic][0]

    def close(self):
        pass


def parse_avro_msg(msg, avro_schema=None) -> dict:
    """Decode a message: Avro binary when a schema is given and the payload is bytes,
    else a JSON-encoded record."""
    v = msg if isinstance(msg, (bytes, str)) else msg.value()
    if isinstance(v, bytes) and avro_schema is not None:
        from . import avro

        return avro.decode(avro_schema, v)
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
