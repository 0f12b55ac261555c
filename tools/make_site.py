"""Static documentation site from the example notebooks.

The reference converts every notebook to markdown with nbconvert, fixes image links and builds a
Hugo site whose index groups pages by category (make.py:15-106;
themes/berbera/layouts/index.html:35-498).  Here the example sources (examples/**.py, the notebook
sources of tools/make_notebooks.py) are rendered directly: markdown cells become prose, code cells
fenced python blocks, one page per example under site/<category>/..., plus site/index.md grouping
pages by top-level category.  Run: python tools/make_site.py [out_dir]
"""
from __future__ import annotations

import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
from make_notebooks import to_cells  # noqa: E402

CATEGORIES = {"ml": "Machine learning", "featurestore": "Feature store", "kafka": "Kafka", "spark": "Streaming & SQL",
              "hive": "Hive"}


def render(src: str) -> tuple[str, str]:
    cells = to_cells(src)
    title = None
    out = []
    for c in cells:
        text = "".join(c["source"])
        if c["cell_type"] == "markdown":
            if title is None:
                for line in text.splitlines():
                    if line.startswith("#"):
                        title = line.lstrip("#").strip()
                        break
            out.append(text)
        else:
            out.append("```python\n" + text + "\n```")
    return title or "untitled", "\n\n".join(out) + "\n"


def build(out_dir: Path) -> list[Path]:
    pages: dict[str, list[tuple[str, str]]] = {}
    written = []
    for p in sorted((ROOT / "examples").rglob("*.py")):
        rel = p.relative_to(ROOT / "examples")
        title, body = render(p.read_text())
        dst = out_dir / rel.with_suffix(".md")
        dst.parent.mkdir(parents=True, exist_ok=True)
        dst.write_text(f"---\ntitle: \"{title}\"\nsource: examples/{rel}\n---\n\n{body}")
        written.append(dst)
        pages.setdefault(rel.parts[0], []).append((title, str(rel.with_suffix(".md"))))
    idx = ["# hopsx examples", ""]
    for cat in sorted(pages, key=lambda c: list(CATEGORIES).index(c) if c in CATEGORIES else 99):
        idx += [f"## {CATEGORIES.get(cat, cat)}", ""]
        idx += [f"* [{t}]({link})" for t, link in sorted(pages[cat])]
        idx.append("")
    (out_dir / "index.md").write_text("\n".join(idx))
    written.append(out_dir / "index.md")
    return written


if __name__ == "__main__":
    out = Path(sys.argv[1]) if len(sys.argv) > 1 else ROOT / "site"
    print(f"wrote {len(build(out))} pages to {out}")
