"""Model registry (``hops.model``): versioned model artifacts under the project's
``Models/<name>/<version>/`` with metrics, used to pick the best model for serving.

Reference: ``model.export(path, name, metrics=…)`` prints
"Exported model <name> as version <v> successfully." and the registry layout
``Models/<name>/<version>/…`` (IrisClassification_And_Serving_SKLearn.ipynb:498-528);
``model.get_best_model(name, metric, Metric.MAX)`` returns
``{'name', 'version', 'metrics': {k: str(v)}}`` (…:547-561, model_repo_and_serving.ipynb:314-335).
"""
from __future__ import annotations

import json
import os
import shutil
import sys
import time
from pathlib import Path

from . import hdfs

META = "model.json"


class Metric:
    MAX = "MAX"
    MIN = "MIN"


class ModelNotFound(Exception):
    pass


def _root() -> Path:
    return Path(hdfs.project_path()) / "Models"


def _versions(name: str) -> list[int]:
    d = _root() / name
    if not d.exists():
        return []
    return sorted(int(p.name) for p in d.iterdir() if p.is_dir() and p.name.isdigit())


def export(model_path: str, model_name: str, model_version: int | None = None, overwrite: bool = False,
           metrics: dict | None = None, description: str | None = None, synchronous: bool = True,
           synchronous_timeout: int = 120, project: str | None = None) -> str:
    """Copy a model file/directory into the registry as a new (or given) version."""
    # a local (cwd-relative) path first, as the reference exports from the executor's local dir,
    # then the project filesystem
    src = Path(model_path) if Path(model_path).exists() else Path(hdfs.abs_path(model_path))
    if not src.exists():
        raise FileNotFoundError(model_path)
    versions = _versions(model_name)
    v = model_version if model_version is not None else (versions[-1] + 1 if versions else 1)
    dest = _root() / model_name / str(v)
    if dest.exists():
        if not overwrite:
            raise IOError(f"model {model_name} version {v} exists (overwrite=False)")
        shutil.rmtree(dest)
    dest.mkdir(parents=True)
    if src.is_dir():
        for item in src.iterdir():
            if item.is_dir():
                shutil.copytree(item, dest / item.name)
            else:
                shutil.copy2(item, dest / item.name)
    else:
        shutil.copy2(src, dest / src.name)
    meta = {
        "name": model_name,
        "version": v,
        "metrics": {k: (float(x) if isinstance(x, (int, float)) else x) for k, x in (metrics or {}).items()},
        "description": description,
        "created": time.time(),
        "experiment_id": os.environ.get("HOPSX_LOGDIR", ""),
        "program": os.path.abspath(sys.argv[0]) if sys.argv and sys.argv[0] else "",
    }
    (dest / META).write_text(json.dumps(meta, indent=2))
    # the reference attaches the generating program; keep a pointer to it
    (dest / "program.txt").write_text(meta["program"] or meta["experiment_id"])
    print(f"Exported model {model_name} as version {v} successfully.")
    return str(dest)


def _meta(name: str, version: int) -> dict:
    p = _root() / name / str(version) / META
    if not p.exists():
        raise ModelNotFound(f"{name} v{version}")
    return json.loads(p.read_text())


def get_model(name: str, version: int) -> dict:
    m = _meta(name, version)
    m["path"] = str(_root() / name / str(version))
    return m


def get_models(name: str | None = None) -> list[dict]:
    names = [name] if name else [p.name for p in _root().iterdir() if p.is_dir()] if _root().exists() else []
    return [get_model(n, v) for n in names for v in _versions(n)]


def get_best_model(name: str, metric: str, direction: str = Metric.MAX) -> dict:
    best = None
    for v in _versions(name):
        m = _meta(name, v)
        val = m["metrics"].get(metric)
        if val is None:
            continue
        val = float(val)
        if best is None or (val > best[0] if direction == Metric.MAX else val < best[0]):
            best = (val, m)
    if best is None:
        raise ModelNotFound(f"no version of {name} has metric {metric!r}")
    m = best[1]
    return {"name": m["name"], "version": m["version"], "metrics": {k: str(v) for k, v in m["metrics"].items()}}


def download_model(name: str, version: int | None = None, local_dir: str = "") -> str:
    v = version if version is not None else _versions(name)[-1]
    return hdfs.copy_to_local(f"Models/{name}/{v}", local_dir or os.getcwd())


def delete(name: str, version: int | None = None) -> None:
    p = _root() / name if version is None else _root() / name / str(version)
    shutil.rmtree(p, ignore_errors=True)


# ----------------------------------------------- torch model save / load helpers
def save_torch(model, path: str, builder: str | None = None, kwargs: dict | None = None) -> str:
    """Save a hopsx/torch model as ``model.pt`` + ``spec.json`` so serving can rebuild it."""
    import torch

    d = Path(path)
    d.mkdir(parents=True, exist_ok=True)
    sd = {k: v.detach().float().cpu() for k, v in model.state_dict().items()}
    torch.save(sd, d / "model.pt")
    spec = {"builder": builder or f"{type(model).__module__}:{type(model).__qualname__}", "kwargs": kwargs or {}}
    (d / "spec.json").write_text(json.dumps(spec))
    return str(d)


def load_torch(path: str, device=None):
    import importlib

    import torch

    d = Path(path)
    spec = json.loads((d / "spec.json").read_text())
    mod, cls = spec["builder"].split(":")
    model = getattr(importlib.import_module(mod), cls)(**spec["kwargs"])
    model.load_state_dict(torch.load(d / "model.pt", weights_only=True, map_location="cpu"))
    model.eval()
    if device is not None:
        model.to(device)
    return model
