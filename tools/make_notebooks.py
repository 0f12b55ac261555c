"""Build notebooks/**.ipynb from examples/**.py (cells split on '# %%'; '# %% [markdown]' cells
become markdown with the leading '# ' stripped).  Run: python tools/make_notebooks.py"""
from __future__ import annotations

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def to_cells(src: str) -> list[dict]:
    cells, cur, kind = [], [], "code"

    def flush():
        text = "\n".join(cur).strip("\n")
        if text:
            if kind == "markdown":
                text = "\n".join(l[2:] if l.startswith("# ") else l.lstrip("#") for l in text.splitlines())
            lines = [l + "\n" for l in text.splitlines()]
            lines[-1] = lines[-1].rstrip("\n")
            cell = {"cell_type": kind, "metadata": {}, "source": lines}
            if kind == "code":
                cell.update(execution_count=None, outputs=[])
            cells.append(cell)

    for line in src.splitlines():
        if line.startswith("# %%"):
            flush()
            cur, kind = [], ("markdown" if "[markdown]" in line else "code")
        else:
            cur.append(line)
    flush()
    return cells


def main() -> int:
    n = 0
    for py in sorted((ROOT / "examples").rglob("*.py")):
        rel = py.relative_to(ROOT / "examples").with_suffix(".ipynb")
        out = ROOT / "notebooks" / rel
        out.parent.mkdir(parents=True, exist_ok=True)
        nb = {"cells": to_cells(py.read_text()), "metadata": {"kernelspec": {"display_name": "Python 3",
                                                                              "language": "python", "name": "python3"},
                                                               "language_info": {"name": "python"}},
              "nbformat": 4, "nbformat_minor": 4}
        out.write_text(json.dumps(nb, indent=1) + "\n")
        n += 1
    print(f"wrote {n} notebooks")
    return 0


if __name__ == "__main__":
    sys.exit(main())
