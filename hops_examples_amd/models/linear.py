"""``LinearClassifier`` over numeric + vocabulary (one-hot indicator) columns, trained
with FTRL — the census income model of the feature-bias notebook
(notebooks/featurestore/feature-bias/feature-bias-whatif.ipynb:46-116 feature columns,
:458-463 ``tf.estimator.LinearClassifier(...).train(steps=5000)``, batch 64).

MI355X mapping: indicator columns are one fixed-length embedding-bag over a single
[sum(vocab sizes) + OOV, 1] weight table (gather fwd / atomic scatter-add bwd), the
numeric part is one MFMA linear, and FTRL is a single fused kernel over the arena.
``predict_proba`` on edited rows gives the What-If-Tool style counterfactuals.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch
from torch import nn

from .. import nn as hnn
from ..ops import functional as HF


class LinearClassifier(nn.Module):
    def __init__(self, numeric: list[str], vocab: dict[str, list]):
        super().__init__()
        self.numeric = list(numeric)
        self.vocab = {k: list(v) for k, v in vocab.items()}
        self._index = {}
        off = 0
        for k, vs in self.vocab.items():
            self._index[k] = (off, {v: i for i, v in enumerate(vs)}, len(vs))
            off += len(vs) + 1  # +1 OOV slot
        self.rows = max(off, 1)
        self.table = nn.Parameter(torch.zeros(self.rows, 1))
        self.dense = hnn.Linear(max(len(self.numeric), 1), 1, init="torch", out_f32=True)
        with torch.no_grad():
            self.dense.weight.zero_()
            self.dense.bias.zero_()
        self.mean = np.zeros(len(self.numeric), np.float32)
        self.std = np.ones(len(self.numeric), np.float32)
        self.device = torch.device("cpu")

    def encode(self, df: pd.DataFrame):
        x = df[self.numeric].to_numpy(np.float32) if self.numeric else np.zeros((len(df), 1), np.float32)
        if self.numeric:
            x = (x - self.mean) / self.std
        cats = []
        for k, (off, m, n) in self._index.items():
            cats.append(np.fromiter((off + m.get(v, n) for v in df[k].tolist()), np.int64, len(df)))
        c = np.stack(cats, 1) if cats else np.zeros((len(df), 0), np.int64)
        return torch.from_numpy(x).to(self.device), torch.from_numpy(c).to(self.device)

    def forward(self, x, c):
        out = self.dense(x if not x.is_cuda else HF.to_compute(x)).float()
        if c.shape[1]:
            out = out + HF.embedding_bag(c, self.table)
        return out

    def fit(self, df: pd.DataFrame, label: str, steps: int = 5000, batch_size: int = 64, lr: float = 0.2,
            device=None, seed: int = 0):
        from .. import optim
        from ..runtime.arena import ParamArena
        from ..runtime.step import TrainStep

        self.device = torch.device(device) if device else (
            torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu"))
        if self.numeric:
            v = df[self.numeric].to_numpy(np.float32)
            self.mean, self.std = v.mean(0), v.std(0) + 1e-6
        self.to(self.device)
        ParamArena.from_module(self, self.device)
        opt = optim.Ftrl(self, lr=lr)
        step = TrainStep(self, opt, "bce_logits", graph=self.device.type == "cuda", forward_fn=lambda m, z: m(*z))
        x, c = self.encode(df)
        y = torch.from_numpy(df[label].to_numpy(np.float32)).to(self.device).view(-1, 1)
        n = len(df)
        g = torch.Generator().manual_seed(seed)
        perm = torch.randperm(n, generator=g).to(self.device)
        losses = []
        for s in range(steps):
            j = (s * batch_size) % max(n - batch_size + 1, 1)
            if j < batch_size and s:
                perm = torch.randperm(n, generator=g).to(self.device)
            idx = perm[j:j + batch_size]
            r = step((x[idx], c[idx]), y[idx])
            if s % 500 == 0 or s == steps - 1:
                losses.append(float(r["loss"].reshape(-1)[0]))
        return losses

    @torch.no_grad()
    def predict_proba(self, df: pd.DataFrame) -> np.ndarray:
        x, c = self.encode(df)
        return torch.sigmoid(self(x, c).float()).cpu().numpy().reshape(-1)

    @torch.no_grad()
    def evaluate(self, df: pd.DataFrame, label: str) -> dict:
        p = self.predict_proba(df)
        y = df[label].to_numpy(np.float32)
        acc = float(((p > 0.5) == (y > 0.5)).mean())
        eps = 1e-7
        loss = float(-(y * np.log(p + eps) + (1 - y) * np.log(1 - p + eps)).mean())
        return {"accuracy": acc, "loss": loss}
