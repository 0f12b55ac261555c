"""Trial-side reporter: metric broadcast + heartbeats to the lagom driver.

Protocol (newline-delimited JSON over a local TCP socket):
  worker -> driver  {"trial": id, "type": "METRIC", "step": s, "value": v}   (heartbeat thread, every hb_interval)
  driver -> worker  {"type": "STOP"}                                          (early stop)
``broadcast`` only records the latest value locally (cheap inside a training
loop); the heartbeat thread ships it, so the GPU step never waits on the driver.
"""
from __future__ import annotations

import json
import os
import socket
import threading
import time


class EarlyStopException(Exception):
    def __init__(self, metric=None):
        super().__init__("trial early-stopped by the lagom driver")
        self.metric = metric


class Reporter:
    def __init__(self, trial_id: str | None = None, host: str | None = None, port: int | None = None,
                 hb_interval: float = 1.0):
        self.trial_id = trial_id or os.environ.get("HOPSX_TRIAL_ID", "local")
        host = host or os.environ.get("HOPSX_MAGGY_HOST")
        port = port or (int(os.environ["HOPSX_MAGGY_PORT"]) if "HOPSX_MAGGY_PORT" in os.environ else None)
        self.hb_interval = float(os.environ.get("HOPSX_MAGGY_HB", hb_interval))
        self.metric = None
        self.step = -1
        self.stop = False
        self.history: list[tuple[int, float]] = []
        self._lock = threading.Lock()
        self._sock = None
        if host and port:
            self._sock = socket.create_connection((host, port), timeout=30)
            self._sock.settimeout(None)
            self._send({"type": "REG"})
            threading.Thread(target=self._hb_loop, daemon=True).start()
            threading.Thread(target=self._rx_loop, daemon=True).start()

    def _send(self, msg: dict):
        if self._sock is None:
            return
        msg["trial"] = self.trial_id
        data = (json.dumps(msg) + "\n").encode()
        with self._lock:
            try:
                self._sock.sendall(data)
            except OSError:
                self._sock = None

    def _hb_loop(self):
        last = None
        while self._sock is not None:
            time.sleep(self.hb_interval)
            if self.metric is not None and (self.step, self.metric) != last:
                last = (self.step, self.metric)
                self._send({"type": "METRIC", "step": self.step, "value": self.metric})

    def _rx_loop(self):
        f = self._sock.makefile("r")
        for line in f:
            try:
                msg = json.loads(line)
            except ValueError:
                continue
            if msg.get("type") == "STOP":
                self.stop = True

    def broadcast(self, metric, step: int | None = None):
        """Report the current metric (called every batch/epoch by the training function)."""
        if hasattr(metric, "item"):
            metric = metric.item()
        self.step = self.step + 1 if step is None else step
        self.metric = float(metric)
        self.history.append((self.step, self.metric))
        if self.stop:
            raise EarlyStopException(self.metric)

    def log(self, msg: str, jupyter: bool = False):
        print(f"[trial {self.trial_id}] {msg}", flush=True)

    def flush(self):
        if self.metric is not None:
            self._send({"type": "METRIC", "step": self.step, "value": self.metric})

    def close(self, final=None):
        self.flush()
        if final is not None:
            self._send({"type": "FINAL", "value": final})
        if self._sock is not None:
            try:
                self._sock.close()
            except OSError:
                pass
            self._sock = None
