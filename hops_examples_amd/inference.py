"""Image inference: single-image prediction and sharded multi-GPU batch inference.

Reference: notebooks/ml/Inference/Inference_Hello_World.ipynb (ResNet50 -> save to the project ->
reload -> ``load_img(target_size=(224, 224))`` -> ``preprocess_input`` -> ``predict`` ->
``decode_predictions(top=3)``) and Batch_Inference_Imagenet_Spark.ipynb (``mapPartitions``
over image paths, 10k-image limit, ``repartition(num_executors * 3)``, Parquet output with
``image_path, top1_label … top3_label``).

MI355X design: instead of Spark executors, ``batch_predict`` shards the image list over one
worker process per GPU; each worker decodes JPEG/PNG on a thread pool (PIL releases the GIL) and
runs a :class:`Predictor`: uint8 NHWC batches are packed into pinned host memory and copied to the
device on a side stream while the previous batch computes (two device input buffers), the forward
+ softmax is replayed from a hipGraph captured once per (batch shape, input buffer) — bf16
ResNet-50 with batch norm in its inference kernel (running statistics + residual + ReLU in one
launch) — and each worker writes its shard as Parquet; the driver concatenates the shards.
No pretrained ImageNet weights exist offline, so models are random-init unless a checkpoint
is loaded, and labels default to ``class_<i>`` (pass ``labels=`` for real names).
"""
from __future__ import annotations

import concurrent.futures as cf
from pathlib import Path

import numpy as np
import pandas as pd

from . import hdfs

HEIGHT = WIDTH = 224


def load_img(path, target_size=(HEIGHT, WIDTH)) -> np.ndarray:
    from PIL import Image

    img = Image.open(str(hdfs._resolve(path)) if not Path(str(path)).exists() else str(path)).convert("RGB")
    if target_size is not None:
        img = img.resize((target_size[1], target_size[0]), Image.BILINEAR)
    return np.asarray(img, dtype=np.uint8)


def img_to_array(img) -> np.ndarray:
    return np.asarray(img, dtype=np.float32)


def preprocess_input(x: np.ndarray) -> np.ndarray:
    """Keras ResNet50 'caffe' preprocessing: RGB->BGR and ImageNet mean subtraction."""
    x = np.asarray(x, dtype=np.float32)[..., ::-1]
    return x - np.array([103.939, 116.779, 123.68], dtype=np.float32)


def decode_predictions(preds, top: int = 3, labels: list[str] | None = None):
    """[(class_id, label, score)] per row, best first (Keras ``decode_predictions`` shape)."""
    preds = np.asarray(preds)
    out = []
    for row in preds:
        idx = np.argsort(-row)[:top]
        out.append([(f"n{i:08d}", labels[i] if labels else f"class_{i}", float(row[i])) for i in idx])
    return out


def _predict_probs(model, x, device):
    import torch

    with torch.no_grad():
        t = torch.from_numpy(np.ascontiguousarray(x)).to(device, non_blocking=True)
        logits = model(t)
        return torch.softmax(logits.float(), dim=-1).cpu().numpy()


class Predictor:
    """Streaming inference on one device.

    ``predict_batches(batches)`` yields softmax probabilities per batch.  On a GPU: batch i+1 is
    packed into a pinned host buffer and copied host->device on a side stream while batch i runs;
    the forward (+ softmax) of each (batch shape, input buffer) pair is captured into a hipGraph on
    first use and replayed afterwards (``graph=False``: eager kernels, same results).  On the CPU
    it is the eager forward."""

    def __init__(self, model, device=None, graph: bool = True):
        import torch

        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu"))
        self.model = model.eval()
        self.cuda = self.device.type == "cuda"
        self.graph = graph and self.cuda
        self._graphs: dict = {}  # (shape, dtype, slot) -> (graph, static_in, static_out)
        self._bufs: dict = {}    # (shape, dtype) -> ([pinned x2], [device x2])
        self._copy = torch.cuda.Stream(self.device) if self.cuda else None
        self.replays = 0

    def _buffers(self, shape, dtype):
        import torch

        key = (tuple(shape), dtype)
        if key not in self._bufs:
            tdt = torch.from_numpy(np.zeros(1, dtype)).dtype
            self._bufs[key] = ([torch.empty(shape, dtype=tdt).pin_memory() for _ in range(2)],
                               [torch.empty(shape, dtype=tdt, device=self.device) for _ in range(2)])
        return self._bufs[key]

    def _forward(self, t):
        import torch

        return torch.softmax(self.model(t).float(), dim=-1)

    def _run(self, dev_in, key):
        import torch

        if not self.graph:
            return self._forward(dev_in)
        g = self._graphs.get(key)
        if g is None:
            from .runtime.capture import graph as capture

            self._forward(dev_in)  # warm-up: first-call allocations and kernel selection, outside capture
            torch.cuda.current_stream(self.device).synchronize()
            cg = torch.cuda.CUDAGraph()
            with capture(cg):
                out = self._forward(dev_in)
            g = self._graphs[key] = (cg, out)
        g[0].replay()
        self.replays += 1
        return g[1]

    def predict_batches(self, batches):
        import torch

        if not self.cuda:
            with torch.no_grad():
                for x in batches:
                    yield self._forward(torch.from_numpy(np.ascontiguousarray(x))).numpy()
            return
        cur = torch.cuda.current_stream(self.device)
        done = [None, None]  # per input slot: event after the last replay that read it

        def stage(x, k):
            """pack batch -> pinned[k], then H2D pinned[k] -> dev[k] on the copy stream once the replay
            that last read dev[k] (two batches ago) has finished."""
            pins, devs = self._buffers(x.shape, x.dtype)
            pins[k].numpy()[...] = x  # pinned[k]'s previous H2D finished before that batch's replay
            if done[k] is not None:
                self._copy.wait_event(done[k])
            with torch.cuda.stream(self._copy):
                devs[k].copy_(pins[k], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self._copy)
            return devs[k], ev, (tuple(x.shape), x.dtype, k)

        it = iter(batches)
        nxt = next(it, None)
        staged = stage(np.ascontiguousarray(nxt), 0) if nxt is not None else None
        slot = 0
        with torch.no_grad():
            while staged is not None:
                dev_in, ev, key = staged
                cur.wait_event(ev)
                out = self._run(dev_in, key)
                done[slot] = torch.cuda.Event()
                done[slot].record(cur)
                nxt = next(it, None)
                slot ^= 1
                # the next batch's packing + H2D overlap this batch's forward
                staged = stage(np.ascontiguousarray(nxt), slot) if nxt is not None else None
                yield out.cpu().numpy()  # the output buffer is reused two batches later


def predict(model, images: np.ndarray, batch_size: int = 64, device=None, graph: bool = True) -> np.ndarray:
    """Softmax probabilities for uint8 NHWC ``images`` (the hopsx ResNets normalise on device)."""
    pr = Predictor(model, device, graph=graph)
    batches = (images[i:i + batch_size] for i in range(0, len(images), batch_size))
    return np.concatenate(list(pr.predict_batches(batches)))


def _shard_worker(model_builder, checkpoint, paths, batch_size, top, labels, out_path, threads):
    import torch

    from .runtime.arena import ParamArena

    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    model = model_builder()
    if checkpoint:
        from .model import load_torch

        sd = load_torch(checkpoint, device="cpu") if str(checkpoint).endswith(".pt") else None
        if isinstance(sd, dict):
            model.load_state_dict(sd)
    model = model.to(dev).eval()
    if dev.type == "cuda":
        ParamArena.from_module(model, dev)
    rows = []
    pool = cf.ThreadPoolExecutor(threads)

    def load(p):
        try:
            return p, load_img(p)
        except Exception:  # malformed images are skipped, as the reference does
            return p, None

    batches = [paths[i:i + batch_size] for i in range(0, len(paths), batch_size)]
    order: list = []  # paths of the batches handed to the predictor, in order

    def decoded():
        fut = pool.map(load, batches[0]) if batches else None
        for bi in range(len(batches)):
            loaded = [(p, a) for p, a in fut if a is not None]
            if bi + 1 < len(batches):
                fut = pool.map(load, batches[bi + 1])  # decode the next batch while this one runs
            if loaded:
                order.append([p for p, _ in loaded])
                yield np.stack([a for _, a in loaded])

    predictor = Predictor(model, dev)
    for bi, probs in enumerate(predictor.predict_batches(decoded())):
        for p, dec in zip(order[bi], decode_predictions(probs, top, labels)):
            r = {"image_path": str(p)}
            for k, (cid, lab, sc) in enumerate(dec, 1):
                r[f"top{k}_id"], r[f"top{k}_label"], r[f"top{k}_score"] = cid, lab, sc
            rows.append(r)
    df = pd.DataFrame(rows)
    if rows:
        df.attrs["graph_replays"] = predictor.replays
    df.to_parquet(out_path, index=False)
    return len(df)


def batch_predict(model_builder, image_paths: list, output_path: str, batch_size: int = 100, top: int = 3,
                  labels: list[str] | None = None, num_workers: int | None = None, limit: int | None = None,
                  checkpoint: str | None = None, decode_threads: int = 8, timeout: float | None = None
                  ) -> pd.DataFrame:
    """Label ``image_paths`` with one worker process per GPU; writes ``output_path`` (Parquet dir)."""
    from .experiment import _runner as R

    paths = list(image_paths)[:limit] if limit else list(image_paths)
    ngpu = R.num_gpus()
    n = num_workers or max(1, ngpu)
    out = Path(hdfs._resolve(output_path))
    out.mkdir(parents=True, exist_ok=True)
    for f in out.glob("part-*.parquet"):
        f.unlink()
    shards = [paths[i::n] for i in range(n)]
    workers = []
    for i, sh in enumerate(shards):
        if not sh:
            continue
        w = R.spawn(_shard_worker, {"model_builder": model_builder, "checkpoint": checkpoint, "paths": sh,
                                    "batch_size": batch_size, "top": top, "labels": labels,
                                    "out_path": str(out / f"part-{i:05d}.parquet"), "threads": decode_threads},
                    out / "_logs", log_name=f"worker_{i}_output.log", gpu=(i % ngpu) if ngpu else None)
        workers.append(w)
    for w in workers:
        R.collect(w, timeout)
    return read_labels(output_path)


def read_labels(output_path: str) -> pd.DataFrame:
    out = Path(hdfs._resolve(output_path))
    frames = [pd.read_parquet(f) for f in sorted(out.glob("part-*.parquet"))]
    return pd.concat(frames, ignore_index=True) if frames else pd.DataFrame()
