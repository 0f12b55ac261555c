"""SVG plotting and the sparkmagic boundary helpers (R15)."""
import xml.etree.ElementTree as ET

import numpy as np
import pandas as pd


def _parse(svg):
    root = ET.fromstring(svg)
    assert root.tag.endswith("svg")
    return root


def test_plots_render_valid_svg(project_root):
    from hops_examples_amd import plotting

    rng = np.random.default_rng(0)
    h = plotting.histogram(rng.normal(size=1000), bins=15, title="hist", xlabel="x")
    r = _parse(h)
    rects = [e for e in r.iter() if e.tag.endswith("rect")]
    assert len(rects) == 16  # background + 15 bins
    _parse(plotting.bar(["a", "b", "c"], [1, -2, 3], title="bars"))
    _parse(plotting.line(np.arange(10), {"loss": np.exp(-np.arange(10) / 3), "acc": np.linspace(0, 1, 10)}))
    _parse(plotting.scatter(rng.normal(size=20000), rng.normal(size=20000), max_points=500))
    corr = pd.DataFrame(rng.normal(size=(100, 4)), columns=list("abcd")).corr()
    _parse(plotting.heatmap(corr.to_numpy(), labels=list(corr.columns), title="corr"))
    g = plotting.geo_heatmap(rng.uniform(59, 60, 500), rng.uniform(17, 19, 500), bins=10)
    assert len([e for e in _parse(g).iter() if e.tag.endswith("rect")]) == 101
    p = plotting.save(h, "Resources/plots/hist.svg")
    assert (project_root / "Resources" / "plots" / "hist.svg").read_text() == h and p.endswith("hist.svg")


def test_sql_magic_binds_output(project_root):
    from hops_examples_amd import hive, notebook

    conn = hive.setup_hive_connection()
    cur = conn.cursor()
    cur.execute("CREATE TABLE sales (store INT, amount DOUBLE) STORED AS ORC")
    cur.execute("INSERT INTO sales VALUES (1, 10.0), (1, 5.0), (2, 7.5)")
    ns = {}
    df = notebook.sql("SELECT store, SUM(amount) AS total FROM sales GROUP BY store ORDER BY store", output="totals",
                      namespace=ns)
    assert ns["totals"] is df and df["total"].tolist() == [15.0, 7.5]
    assert notebook.local(lambda a: a + 1, 1) == 2
    assert notebook.Session().info()["State"] == "idle"


def test_make_site(tmp_path):
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))
    import make_site

    pages = make_site.build(tmp_path)
    idx = (tmp_path / "index.md").read_text()
    assert "## Feature store" in idx and "## Machine learning" in idx and len(pages) > 20
    md = (tmp_path / "featurestore" / "tour" / "featurestore_tour_job.md").read_text()
    assert md.startswith("---\ntitle: \"Feature store tour: feature engineering job\"") and "```python" in md
