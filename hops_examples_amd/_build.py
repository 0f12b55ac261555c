"""In-tree native build for the hopsx extensions (no JIT cache, no hipify).

* ``_hopsx_ops``  — HIP/CDNA4 kernel library (csrc/ops/*.hip + bindings.cpp), gfx950 only.
* ``_hopsx_io``   — C++ data path: TFRecord/CSV codecs, shard planner, pinned
                    staging ring (csrc/io/*.cpp).
* ``_hopsx_comm`` — C++/HIP communication helpers: one-shot xGMI all-reduce over
                    IPC-mapped peer buffers, bucket planner (csrc/comm/*).

Objects are cached under ``build/`` and rebuilt when a source or any header in
its directory is newer.  The resulting ``.so`` files live next to this file so
that ``gpurun`` snapshots carry them to the GPU box.

Usage: ``python -m hops_examples_amd._build [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import hashlib
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "hops_examples_amd"
BUILD = ROOT / "build"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _py_includes() -> list[str]:
    import pybind11

    return ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"]]


def _newer(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps if d.exists())


def _digest(cmd: list[str], deps: list[Path]) -> str:
    """Content hash of the compile command and every input: an object is reused only when it was
    built from exactly these bytes (mtimes alone miss a source edited while a build was running)."""
    h = hashlib.sha1(" ".join(cmd).encode())
    for d in deps:
        if d.exists():
            h.update(d.name.encode())
            h.update(d.read_bytes())
    return h.hexdigest()


def _stale(o: Path, cmd: list[str], deps: list[Path]) -> tuple[bool, str]:
    dg = _digest(cmd, deps)
    stamp = o.with_suffix(o.suffix + ".sha1")
    return (not o.exists() or not stamp.exists() or stamp.read_text().strip() != dg), dg


def _local_includes(src: Path, search: list[Path], seen: set | None = None) -> list[Path]:
    """Transitive ``#include "x.h"`` headers of a source found in ``search`` (the rebuild digest of
    an object covers exactly what it includes: editing one kernel's header no longer rebuilds every
    translation unit)."""
    seen = set() if seen is None else seen
    out = []
    try:
        text = src.read_text(errors="ignore")
    except OSError:
        return out
    for ln in text.splitlines():
        ln = ln.strip()
        if not ln.startswith("#include") or '"' not in ln:
            continue
        name = ln.split('"')[1]
        for d in [src.parent, *search]:
            h = d / name
            if h.exists():
                if h not in seen:
                    seen.add(h)
                    out.append(h)
                    out.extend(_local_includes(h, search, seen))
                break
    return out


def _check_undefined(lib: Path) -> None:
    """A symbol of our own left undefined in the extension would only fail when first called (lazy
    binding aborts the process): refuse such a link."""
    r = subprocess.run(["nm", "-D", "--undefined-only", str(lib)], stdout=subprocess.PIPE, text=True)
    bad = [ln.split()[-1] for ln in r.stdout.splitlines() if ln.split() and ln.split()[-1].startswith("hopsx_")]
    if bad:
        lib.unlink()
        raise RuntimeError(f"{lib.name}: undefined hopsx symbols {bad}")


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)


HIP_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-fPIC",
    "-std=c++17",
    "-ffp-contract=fast",
    "-Wno-unused-result",
    "-Wno-unused-variable",
]


def _build_lib(name: str, srcdir: Path, kind: str, force: bool, jobs: int, extra_link: list[str],
               extra_headers: list[Path] | None = None, defines: list[str] | None = None) -> Path:
    """kind: 'hip' compiles every source with hipcc for gfx950, 'cpp' with g++.  ``extra_headers``:
    headers outside ``srcdir`` the sources include (part of the rebuild digest).  ``defines``: extra
    -D flags of the HIP compiles (the debug variant)."""
    out = PKG / f"{name}{EXT}"
    objdir = BUILD / name
    objdir.mkdir(parents=True, exist_ok=True)
    srcs = sorted([*srcdir.glob("*.hip"), *srcdir.glob("*.cpp")])
    headers = sorted(srcdir.glob("*.h")) + list(extra_headers or [])
    jobs_list = []
    for s in srcs:
        o = objdir / (s.name + ".o")
        if kind == "hip" or s.suffix == ".hip":
            cmd = [HIPCC, *HIP_FLAGS, *(defines or []), *_py_includes(), f"-I{srcdir}", "-c", str(s), "-o", str(o)]
            if s.suffix == ".cpp":
                cmd.insert(1, "-x")
                cmd.insert(2, "hip")
        else:
            cmd = ["g++", "-O3", "-fPIC", "-std=c++17", "-march=x86-64-v2", "-msse4.2", "-pthread",
                   *_py_includes(), f"-I{srcdir}", "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__",
                   "-c", str(s), "-o", str(o)]
        # the digest is taken BEFORE compiling: an edit during the compile leaves a mismatching stamp
        deps = _local_includes(s, [srcdir, *{h.parent for h in headers}])
        stale, dg = _stale(o, cmd, [s, *sorted(set(deps) | set(extra_headers or []))])
        if force or stale:
            jobs_list.append((cmd, o, dg))

    def _compile(job):
        cmd, o, dg = job
        _run(cmd)
        o.with_suffix(o.suffix + ".sha1").write_text(dg)

    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            list(ex.map(_compile, jobs_list))
    objs = [str(objdir / (s.name + ".o")) for s in srcs]
    if force or jobs_list or _newer(out, [Path(o) for o in objs]):
        if kind == "hip":
            cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", str(out), *extra_link]
        else:
            cmd = ["g++", "-shared", "-fPIC", "-pthread", *objs, "-o", str(out), *extra_link]
        _run(cmd)
        _check_undefined(out)
    return out


def build(force: bool = False, jobs: int | None = None, verbose: bool = True, debug: bool = False) -> list[Path]:
    """The three in-tree extensions; ``debug=True`` also builds ``_hopsx_ops_dbg``, the kernel library
    with the device-side bound checks compiled in (common.h hx_check; loaded when HOPSX_DEBUG=1)."""
    jobs = jobs or min(8, os.cpu_count() or 4)
    outs = []
    outs.append(_build_lib("_hopsx_ops", ROOT / "csrc" / "ops", "hip", force, jobs, []))
    if debug:
        outs.append(_build_lib("_hopsx_ops_dbg", ROOT / "csrc" / "ops", "hip", force, jobs, [],
                               defines=["-DHOPSX_DEBUG=1", "-DHOPSX_MODNAME=_hopsx_ops_dbg"]))
    if (ROOT / "csrc" / "io").exists() and any((ROOT / "csrc" / "io").glob("*.cpp")):
        outs.append(_build_lib("_hopsx_io", ROOT / "csrc" / "io", "cpp", force, jobs,
                               []))
    if (ROOT / "csrc" / "comm").exists() and any((ROOT / "csrc" / "comm").glob("*.hip")):
        # the fused data-parallel step shares the optimizer update rules with csrc/ops
        outs.append(_build_lib("_hopsx_comm", ROOT / "csrc" / "comm", "hip", force, jobs, [],
                               [ROOT / "csrc" / "ops" / "optim_core.h", ROOT / "csrc" / "ops" / "common.h"]))
    if verbose:
        for o in outs:
            print(f"[hopsx build] {o.relative_to(ROOT)} ({o.stat().st_size // 1024} KiB)")
    return outs


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--debug", action="store_true", help="also build _hopsx_ops_dbg (device bound checks)")
    a = ap.parse_args()
    try:
        build(force=a.force, jobs=a.j, debug=a.debug)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
