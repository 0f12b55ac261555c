"""Image inference: single-image prediction and sharded multi-GPU batch inference.

Reference: notebooks/ml/Inference/Inference_Hello_World.ipynb (ResNet50 -> save to the project ->
reload -> ``load_img(target_size=(224, 224))`` -> ``preprocess_input`` -> ``predict`` ->
``decode_predictions(top=3)``) and Batch_Inference_Imagenet_Spark.ipynb (``mapPartitions``
over image paths, 10k-image limit, ``repartition(num_executors * 3)``, Parquet output with
``image_path, top1_label … top3_label``).

MI355X design: instead of Spark executors, ``batch_predict`` shards the image list over one
worker process per GPU; each worker decodes JPEG/PNG on a thread pool (PIL releases the GIL),
packs uint8 NHWC batches into pinned memory, copies them on a side stream while the previous
batch runs (bf16 ResNet-50 forward, BN folded to inference kernels, whole forward captured in a
hipGraph per batch shape), and writes its shard as Parquet; the driver concatenates the shards.
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


def predict(model, images: np.ndarray, batch_size: int = 64, device=None) -> np.ndarray:
    """Softmax probabilities for uint8 NHWC ``images`` (the hopsx ResNets normalise on device)."""
    import torch

    device = device or (torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu"))
    model.eval()
    return np.concatenate([_predict_probs(model, images[i:i + batch_size], device)
                           for i in range(0, len(images), batch_size)])


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
    fut = pool.map(load, batches[0]) if batches else None
    for bi in range(len(batches)):
        loaded = [(p, a) for p, a in fut if a is not None]
        if bi + 1 < len(batches):
            fut = pool.map(load, batches[bi + 1])  # decode the next batch while this one runs
        if not loaded:
            continue
        x = np.stack([a for _, a in loaded])
        probs = _predict_probs(model, x, dev)
        for (p, _), dec in zip(loaded, decode_predictions(probs, top, labels)):
            r = {"image_path": str(p)}
            for k, (cid, lab, sc) in enumerate(dec, 1):
                r[f"top{k}_id"], r[f"top{k}_label"], r[f"top{k}_score"] = cid, lab, sc
            rows.append(r)
    df = pd.DataFrame(rows)
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
