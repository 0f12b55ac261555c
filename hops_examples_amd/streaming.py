"""Micro-batch streaming from project topics to file sinks with checkpointed offsets
(Structured-Streaming-shaped: notebooks/spark/KafkaSparkPython.ipynb:293-334 readStream from Kafka
-> CSV sink with ``checkpointLocation``; spark/…/StructuredStreamingKafka.scala:22-41 Avro
consumer -> Parquet sink; …/KafkaSparkPython_ConsumeDemoProducer.ipynb text sink).

    q = (streaming.read_stream("test", starting_offsets="earliest")
            .select(lambda df: df.assign(v=df.value.astype(float)))     # any pandas transform
            .write_stream(format="csv", path="Resources/out", checkpoint_location="Resources/ckpt",
                          trigger_interval=0.5)
            .start())
    q.process_all_available(); q.stop()

Exactly-once file output: each micro-batch writes ``part-<batch>.<ext>`` then commits the
next offset to ``<checkpoint>/offsets.json``; a restarted query resumes from the commit and
re-writes (overwrites) a batch that was written but not committed.
"""
from __future__ import annotations

import json
import threading
import time
from pathlib import Path

import pandas as pd

from . import hdfs, kafka


class StreamReader:
    def __init__(self, topic: str, starting_offsets: str = "earliest", value_format: str = "raw",
                 avro_schema=None, max_offsets_per_trigger: int | None = None):
        self.topic, self.start, self.fmt = topic, starting_offsets, value_format
        self.schema = avro_schema
        self.max = max_offsets_per_trigger
        self.transforms = []

    def select(self, fn) -> "StreamReader":
        self.transforms.append(fn)
        return self

    map_batches = select

    def from_avro(self, schema=None) -> "StreamReader":
        self.fmt, self.schema = "avro", schema or kafka.get_schema(self.topic)
        return self

    def from_json(self) -> "StreamReader":
        self.fmt = "json"
        return self

    def write_stream(self, format: str = "csv", path: str | None = None, checkpoint_location: str | None = None,
                     trigger_interval: float = 1.0, output_mode: str = "append", header: bool = True,
                     foreach_batch=None) -> "StreamingQuery":
        return StreamingQuery(self, format, path, checkpoint_location, trigger_interval, header, foreach_batch)

    writeStream = write_stream  # noqa: N815


def read_stream(topic: str, starting_offsets: str = "earliest", **kw) -> StreamReader:
    return StreamReader(topic, starting_offsets, **kw)


class StreamingQuery:
    def __init__(self, reader: StreamReader, fmt, path, ckpt, interval, header, foreach_batch):
        if fmt != "console" and foreach_batch is None and path is None:
            raise ValueError("a file sink needs path=")
        if ckpt is None:
            raise ValueError("checkpoint_location is required")
        self.r, self.fmt, self.interval, self.header = reader, fmt, interval, header
        self.path = Path(hdfs._resolve(path)) if path else None
        self.ckpt = Path(hdfs._resolve(ckpt))
        self.foreach = foreach_batch
        self._stop = threading.Event()
        self._thread = None
        self._lock = threading.Lock()
        self.batches = 0
        self.exception: Exception | None = None

    # ---------------------------------------------------------------- state
    def _load(self):
        p = self.ckpt / "offsets.json"
        if p.exists():
            return json.loads(p.read_text())
        start = 0 if self.r.start == "earliest" else kafka.end_offset(self.r.topic)
        return {"next_offset": start, "next_batch": 0}

    def _commit(self, st):
        self.ckpt.mkdir(parents=True, exist_ok=True)
        tmp = self.ckpt / "offsets.json.tmp"
        tmp.write_text(json.dumps(st))
        tmp.replace(self.ckpt / "offsets.json")

    # ---------------------------------------------------------------- batches
    def _fetch(self, start: int):
        p = kafka.topic_path(self.r.topic)
        if not p.exists():
            return [], start
        rows = []
        with open(p, "rb") as f:
            for i, line in enumerate(f):
                if i < start:
                    continue
                if not line.endswith(b"\n"):
                    break
                if self.r.max is not None and len(rows) >= self.r.max:
                    break
                rec = json.loads(line)
                m = kafka.Message(self.r.topic, rec, i)
                v = m.value()
                if self.r.fmt == "avro":
                    row = kafka.parse_avro_msg(v, self.r.schema)
                elif self.r.fmt == "json":
                    row = json.loads(v) if isinstance(v, (str, bytes)) else v
                else:
                    row = {"key": m.key(), "value": v.decode() if isinstance(v, bytes) else v}
                row = dict(row)
                row.setdefault("offset", i)
                row.setdefault("timestamp", pd.Timestamp(rec["timestamp"], unit="s"))
                rows.append(row)
        return rows, start + len(rows)

    def _write(self, df: pd.DataFrame, batch: int):
        if self.foreach is not None:
            self.foreach(df, batch)
            return
        if self.fmt == "console":
            print(f"Batch: {batch}\n{df.to_string(index=False)}", flush=True)
            return
        self.path.mkdir(parents=True, exist_ok=True)
        name = self.path / f"part-{batch:05d}"
        if self.fmt == "csv":
            df.to_csv(f"{name}.csv", index=False, header=self.header)
        elif self.fmt == "parquet":
            df.to_parquet(f"{name}.parquet", index=False)
        elif self.fmt == "text":
            Path(f"{name}.txt").write_text("\n".join(map(str, df.iloc[:, 0].tolist())) + "\n")
        elif self.fmt == "json":
            df.to_json(f"{name}.json", orient="records", lines=True)
        else:
            raise ValueError(f"unknown sink format {self.fmt}")

    def run_once(self) -> int:
        """Process one micro-batch; returns the number of records consumed."""
        with self._lock:
            st = self._load()
            rows, nxt = self._fetch(st["next_offset"])
            if not rows:
                return 0
            df = pd.DataFrame(rows)
            for fn in self.r.transforms:
                df = fn(df)
            self._write(df, st["next_batch"])
            self._commit({"next_offset": nxt, "next_batch": st["next_batch"] + 1})
            self.batches += 1
            return len(rows)

    def _loop(self):
        try:
            while not self._stop.is_set():
                if self.run_once() == 0:
                    self._stop.wait(self.interval)
        except Exception as e:  # surfaced by awaitTermination / status
            self.exception = e

    def start(self) -> "StreamingQuery":
        self._thread = threading.Thread(target=self._loop, daemon=True)
        self._thread.start()
        return self

    def process_all_available(self, timeout: float = 60.0):
        end = kafka.end_offset(self.r.topic)
        t0 = time.time()
        while self._load()["next_offset"] < end:
            if self.exception:
                raise self.exception
            if self._thread is None:
                self.run_once()
            elif time.time() - t0 > timeout:
                raise TimeoutError("stream did not catch up")
            else:
                time.sleep(0.01)

    processAllAvailable = process_all_available  # noqa: N815

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(10)

    def await_termination(self, timeout: float | None = None) -> bool:
        if self._thread is not None:
            self._thread.join(timeout)
        if self.exception:
            raise self.exception
        return not (self._thread and self._thread.is_alive())

    awaitTermination = await_termination  # noqa: N815

    @property
    def is_active(self) -> bool:
        return bool(self._thread and self._thread.is_alive())

    @property
    def status(self) -> dict:
        st = self._load()
        return {"isActive": self.is_active, "batchesProcessed": self.batches, **st}


def read_sink(path: str, fmt: str = "csv") -> pd.DataFrame:
    p = Path(hdfs._resolve(path))
    files = sorted(p.glob(f"part-*.{ {'text': 'txt'}.get(fmt, fmt) }"))
    if fmt == "csv":
        frames = [pd.read_csv(f) for f in files]
    elif fmt == "parquet":
        frames = [pd.read_parquet(f) for f in files]
    elif fmt == "json":
        frames = [pd.read_json(f, lines=True) for f in files]
    else:
        frames = [pd.DataFrame({"value": f.read_text().splitlines()}) for f in files]
    return pd.concat(frames, ignore_index=True) if frames else pd.DataFrame()
