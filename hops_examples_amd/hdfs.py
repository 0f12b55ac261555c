"""Project filesystem — the hopsx stand-in for HopsFS (``hops.hdfs``).

Reference surface: notebooks/ml/Filesystem/HopsFSOperations.ipynb:62-281 and
the call sites listed in SURVEY.md Appendix A.2.  A *project* is a directory
(``HOPSX_PROJECT_ROOT``) with the standard Hopsworks datasets
(Resources/, Logs/, Experiments/, Models/, Jupyter/, TourData/).  Paths are
resolved like HopsFS paths: relative paths are relative to the project root,
``hdfs://…/Projects/<p>/x`` and ``hopsfs://…`` URIs map onto it, absolute local
paths pass through.
"""
from __future__ import annotations

import fnmatch
import glob as _glob
import os
import shutil
import stat as _stat
from pathlib import Path

from . import config

DATASETS = ("Resources", "Logs", "Experiments", "Models", "Jupyter", "TourData", "Training_Datasets")


def _root() -> Path:
    r = config.get().project_root
    for d in DATASETS:
        (r / d).mkdir(parents=True, exist_ok=True)
    return r


def project_name() -> str:
    return config.get().project_name


def project_user() -> str:
    return f"{config.get().project_name}__{config.get().user}"


def project_id() -> int:
    return abs(hash(config.get().project_name)) % 100000


def project_path(project: str | None = None, exclude_nn_addr: bool = False) -> str:
    """Absolute path of the project root with a trailing separator."""
    if project is None or project == project_name():
        return str(_root()) + os.sep
    p = _root().parent / project
    p.mkdir(parents=True, exist_ok=True)
    return str(p) + os.sep


def get_plain_path(path: str) -> str:
    return str(_resolve(path))


def _resolve(path) -> Path:
    s = str(path)
    for pre in ("hdfs://", "hopsfs://", "file://"):
        if s.startswith(pre):
            rest = s[len(pre):]
            if "/Projects/" in rest:
                rest = rest.split("/Projects/", 1)[1]
                parts = rest.split("/", 1)
                proj = parts[0]
                sub = parts[1] if len(parts) > 1 else ""
                base = Path(project_path(proj))
                return base / sub
            s = "/" + rest.lstrip("/") if pre == "file://" else rest
            break
    p = Path(s)
    if p.is_absolute():
        return p
    return _root() / p


def abs_path(path: str) -> str:
    return str(_resolve(path))


def exists(path: str) -> bool:
    return _resolve(path).exists()


def isdir(path: str) -> bool:
    return _resolve(path).is_dir()


def isfile(path: str) -> bool:
    return _resolve(path).is_file()


def load(path: str) -> bytes:
    return _resolve(path).read_bytes()


def dump(data, path: str) -> None:
    p = _resolve(path)
    p.parent.mkdir(parents=True, exist_ok=True)
    if isinstance(data, str):
        data = data.encode()
    p.write_bytes(data)


def mkdir(path: str) -> None:
    _resolve(path).mkdir(parents=True, exist_ok=True)


def ls(path: str = "", recursive: bool = False, exclude_nn_addr: bool = False) -> list[str]:
    p = _resolve(path)
    if not p.exists():
        raise IOError(f"path does not exist: {path}")
    if p.is_file():
        return [str(p)]
    it = p.rglob("*") if recursive else p.iterdir()
    return sorted(str(x) for x in it)


def lsl(path: str = "", recursive: bool = False) -> list[dict]:
    out = []
    for f in ls(path, recursive):
        st = os.stat(f)
        out.append({"name": f, "kind": "directory" if os.path.isdir(f) else "file", "size": st.st_size,
                    "permissions": _stat.filemode(st.st_mode), "last_mod": st.st_mtime, "owner": project_user()})
    return out


def glob(pattern: str) -> list[str]:
    return sorted(_glob.glob(str(_resolve(pattern))))


def cp(src: str, dest: str, overwrite: bool = False) -> None:
    s, d = _resolve(src), _resolve(dest)
    if d.exists() and not overwrite:
        raise IOError(f"destination exists: {dest}")
    d.parent.mkdir(parents=True, exist_ok=True)
    if s.is_dir():
        if d.exists():
            shutil.rmtree(d)
        shutil.copytree(s, d)
    else:
        shutil.copy2(s, d)


def move(src: str, dest: str) -> None:
    d = _resolve(dest)
    d.parent.mkdir(parents=True, exist_ok=True)
    shutil.move(str(_resolve(src)), str(d))


rename = move


def rmr(path: str, recursive: bool = True) -> None:
    p = _resolve(path)
    if p.is_dir():
        shutil.rmtree(p)
    elif p.exists():
        p.unlink()


def rm(path: str, recursive: bool = False) -> None:
    rmr(path, recursive)


def chmod(path: str, mode: int) -> None:
    os.chmod(_resolve(path), mode)


def chown(path: str, user: str, group: str) -> None:
    # project-level ownership is recorded, not enforced (single-user local project)
    meta = _resolve(path)
    if not meta.exists():
        raise IOError(path)


def stat(path: str) -> os.stat_result:
    return os.stat(_resolve(path))


def access(path: str, mode: int) -> bool:
    return os.access(_resolve(path), mode)


def copy_to_hdfs(local_path: str, hdfs_path: str = "", overwrite: bool = False) -> str:
    """Copy a local file/dir INTO the project directory ``hdfs_path``."""
    src = Path(local_path)
    dest_dir = _resolve(hdfs_path)
    dest_dir.mkdir(parents=True, exist_ok=True)
    dest = dest_dir / src.name
    if dest.exists():
        if not overwrite:
            raise IOError(f"{dest} exists (overwrite=False)")
        rmr(str(dest))
    if src.is_dir():
        shutil.copytree(src, dest)
    else:
        shutil.copy2(src, dest)
    return str(dest)


def copy_to_local(hdfs_path: str, local_path: str = "", overwrite: bool = False, project: str | None = None) -> str:
    """Copy a project file/dir to the local working dir; returns the local dir with a trailing sep
    (``hdfs.copy_to_local('TourData/mnist/MNIST')`` in notebooks/ml/Experiment/PyTorch/mnist.ipynb:190)."""
    src = _resolve(hdfs_path)
    base = Path(local_path) if local_path else Path(os.getcwd())
    base.mkdir(parents=True, exist_ok=True)
    dest = base / src.name
    if dest.exists() and overwrite:
        rmr(str(dest))
    if not dest.exists():
        if src.is_dir():
            shutil.copytree(src, dest)
        else:
            shutil.copy2(src, dest)
    return str(base) + os.sep


class _FS:
    def open_file(self, path, mode="rb", flags=None, **kw):
        p = _resolve(path)
        if any(c in mode for c in "wa"):
            p.parent.mkdir(parents=True, exist_ok=True)
        m = mode.replace("t", "")
        if "b" not in m and "t" not in mode:
            m = m
        return open(p, m if m else "r")

    def exists(self, path):
        return exists(path)

    def ls(self, path):
        return ls(path)

    def delete(self, path, recursive=False):
        rmr(path)


def get_fs() -> _FS:
    return _FS()


def open_file(path: str, project: str | None = None, mode: str = "r", **kw):
    return _FS().open_file(path, mode)


def localize(path: str) -> str:
    return copy_to_local(path)


def find(pattern: str, path: str = "") -> list[str]:
    base = _resolve(path)
    return sorted(str(p) for p in base.rglob("*") if fnmatch.fnmatch(p.name, pattern))
