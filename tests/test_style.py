"""Source style / policy gate — the role of the reference's checkstyle run in Maven's validate phase
(tools/maven/checkstyle.xml:6-51, pom.xml:128-149), applied to this repo's Python and HIP/C++ sources.

Besides layout rules (line length, tabs, trailing whitespace) it enforces the framework's
MI355X-only policy: no CUDA headers or runtime calls, no dual-platform #ifdefs, no hipify
output, and no scalar-cache stores in device code."""
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
try:
    import tomllib
except ImportError:  # python 3.10
    import tomli as tomllib

MAXLEN = tomllib.loads((ROOT / "pyproject.toml").read_text())["tool"]["hopsx"]["style"]["max_line_length"]


def _tracked(*globs):
    out = subprocess.run(["git", "ls-files", *globs], cwd=ROOT, capture_output=True, text=True)
    if out.returncode != 0:  # not a git checkout: walk the tree
        return sorted(p for g in globs for p in ROOT.rglob(g) if ".git" not in p.parts)
    return [ROOT / f for f in out.stdout.split()]


PY = _tracked("*.py")
NATIVE = _tracked("*.hip", "*.cpp", "*.h", "*.hpp")


def test_layout_rules():
    bad = []
    for f in PY + NATIVE:
        for i, line in enumerate(f.read_text(errors="replace").splitlines(), 1):
            if len(line) > MAXLEN:
                bad.append(f"{f.relative_to(ROOT)}:{i}: line longer than {MAXLEN}")
            if "\t" in line and f.suffix == ".py":
                bad.append(f"{f.relative_to(ROOT)}:{i}: tab")
            if line != line.rstrip():
                bad.append(f"{f.relative_to(ROOT)}:{i}: trailing whitespace")
    assert not bad, "\n".join(bad[:50])


POLICY = [
    (re.compile(r"#\s*include\s*[<\"]cuda"), "CUDA header"),
    (re.compile(r"\bcuda(Malloc|Memcpy|Stream|Launch|DeviceSynchronize)\w*\s*\("), "CUDA runtime call"),
    (re.compile(r"__HIP_PLATFORM_(AMD|NVIDIA|NVCC)__"), "dual-platform #ifdef"),
    (re.compile(r"HIPIFY|hipify", re.I), "hipify output"),
    (re.compile(r"\bs_(buffer_|scratch_)?store_dword|\bs_dcache_(wb|discard)|\bs_atomic_"),
     "scalar-cache store in device code"),
]


@pytest.mark.parametrize("path", NATIVE, ids=lambda p: str(p.relative_to(ROOT)))
def test_native_sources_are_mi355x_only(path):
    text = path.read_text(errors="replace")
    hits = [(why, text[:m.start()].count("\n") + 1) for rx, why in POLICY for m in rx.finditer(text)]
    assert not hits, f"{path.relative_to(ROOT)}: {hits}"


def test_native_sources_exist():
    assert any(p.suffix == ".hip" for p in NATIVE) and any(p.suffix == ".cpp" for p in NATIVE)
