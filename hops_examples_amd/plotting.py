"""Plotting without a display stack.

The reference's plotting notebooks pull query results to the driver and draw them with
seaborn/matplotlib (notebooks/ml/Plotting/matplotlib_sparkmagic.ipynb:194-1309), folium heat maps
(…/folium_heat_map.ipynb:37-111) and ipyleaflet (…/ipyleaflet.ipynb:21-251).  None of those
libraries is part of this stack, so charts are rendered here as self-contained SVG documents (any
browser, TensorBoard text plugin or notebook renders them) from pandas / numpy / torch data:

* :func:`histogram`, :func:`bar`, :func:`line`, :func:`scatter`, :func:`heatmap` (e.g. the
  feature-correlation matrix of ``featurestore.statistics``), :func:`geo_heatmap` (lat/lon point
  density binned onto a grid, the folium HeatMap use case);
* ``save(svg, path)`` writes into the project (``hdfs`` paths accepted).

Binning of large inputs (histograms, geo densities) runs through numpy / torch reductions; the SVG
writer only ever sees the binned counts.
"""
from __future__ import annotations

import html
import math
from pathlib import Path

import numpy as np

_W, _H, _PAD = 640, 400, 48
_COLORS = ["#1f77b4", "#ff7f0e", "#2ca02c", "#d62728", "#9467bd", "#8c564b", "#e377c2", "#7f7f7f"]


def _arr(x) -> np.ndarray:
    if hasattr(x, "detach"):
        x = x.detach().float().cpu().numpy()
    return np.asarray(x, dtype=np.float64).ravel()


def _svg(body: list[str], title: str, w=_W, h=_H) -> str:
    t = f'<text x="{w / 2}" y="20" text-anchor="middle" font-size="15">{html.escape(title)}</text>' if title else ""
    return (f'<svg xmlns="http://www.w3.org/2000/svg" width="{w}" height="{h}" viewBox="0 0 {w} {h}" '
            f'font-family="sans-serif">\n<rect width="{w}" height="{h}" fill="white"/>\n{t}\n' + "\n".join(body)
            + "\n</svg>\n")


def _nice(v: float) -> str:
    if v == 0:
        return "0"
    a = abs(v)
    return f"{v:.3g}" if 1e-3 <= a < 1e5 else f"{v:.2e}"


class _Axes:
    def __init__(self, xlo, xhi, ylo, yhi, w=_W, h=_H):
        if xhi <= xlo:
            xhi = xlo + 1.0
        if yhi <= ylo:
            yhi = ylo + 1.0
        self.xlo, self.xhi, self.ylo, self.yhi, self.w, self.h = xlo, xhi, ylo, yhi, w, h

    def x(self, v):
        return _PAD + (v - self.xlo) / (self.xhi - self.xlo) * (self.w - 2 * _PAD)

    def y(self, v):
        return self.h - _PAD - (v - self.ylo) / (self.yhi - self.ylo) * (self.h - 2 * _PAD)

    def frame(self, xlabel="", ylabel="", ticks=5) -> list[str]:
        b = [f'<line x1="{_PAD}" y1="{self.h - _PAD}" x2="{self.w - _PAD}" y2="{self.h - _PAD}" stroke="black"/>',
             f'<line x1="{_PAD}" y1="{_PAD}" x2="{_PAD}" y2="{self.h - _PAD}" stroke="black"/>']
        for i in range(ticks + 1 if ticks > 0 else 0):
            xv = self.xlo + (self.xhi - self.xlo) * i / ticks
            yv = self.ylo + (self.yhi - self.ylo) * i / ticks
            b.append(f'<text x="{self.x(xv):.1f}" y="{self.h - _PAD + 14}" text-anchor="middle" '
                     f'font-size="10">{_nice(xv)}</text>')
            b.append(f'<text x="{_PAD - 4}" y="{self.y(yv) + 3:.1f}" text-anchor="end" font-size="10">'
                     f'{_nice(yv)}</text>')
        if xlabel:
            b.append(f'<text x="{self.w / 2}" y="{self.h - 8}" text-anchor="middle" font-size="12">'
                     f'{html.escape(xlabel)}</text>')
        if ylabel:
            b.append(f'<text x="12" y="{self.h / 2}" text-anchor="middle" font-size="12" '
                     f'transform="rotate(-90 12 {self.h / 2})">{html.escape(ylabel)}</text>')
        return b


def histogram(values, bins: int = 20, title: str = "", xlabel: str = "", range=None) -> str:  # noqa: A002
    v = _arr(values)
    v = v[np.isfinite(v)]
    counts, edges = np.histogram(v, bins=bins, range=range)
    ax = _Axes(edges[0], edges[-1], 0, max(1, counts.max()) * 1.05)
    body = ax.frame(xlabel, "count")
    for c, a, b in zip(counts, edges[:-1], edges[1:]):
        body.append(f'<rect x="{ax.x(a):.1f}" y="{ax.y(c):.1f}" width="{max(ax.x(b) - ax.x(a) - 1, 0.5):.1f}" '
                    f'height="{ax.y(0) - ax.y(c):.1f}" fill="{_COLORS[0]}"/>')
    return _svg(body, title)


def bar(labels, values, title: str = "", ylabel: str = "") -> str:
    v = _arr(values)
    n = len(v)
    ax = _Axes(0, n, min(0.0, v.min()) if n else 0, (v.max() if n else 1) * 1.05)
    body = ax.frame("", ylabel, ticks=0)
    for i, (lab, val) in enumerate(zip(labels, v)):
        x0, x1 = ax.x(i + 0.1), ax.x(i + 0.9)
        top, base = ax.y(max(val, 0)), ax.y(min(val, 0))
        body.append(f'<rect x="{x0:.1f}" y="{top:.1f}" width="{x1 - x0:.1f}" height="{base - top:.1f}" '
                    f'fill="{_COLORS[i % len(_COLORS)]}"/>')
        body.append(f'<text x="{(x0 + x1) / 2:.1f}" y="{_H - _PAD + 14}" text-anchor="middle" font-size="10">'
                    f'{html.escape(str(lab))[:12]}</text>')
    return _svg(body, title)


def line(x, ys: dict | list, title: str = "", xlabel: str = "", ylabel: str = "") -> str:
    xa = _arr(x)
    series = ys if isinstance(ys, dict) else {"": ys}
    arrs = {k: _arr(v) for k, v in series.items()}
    allv = np.concatenate(list(arrs.values())) if arrs else np.zeros(1)
    ax = _Axes(xa.min(), xa.max(), float(np.nanmin(allv)), float(np.nanmax(allv)))
    body = ax.frame(xlabel, ylabel)
    for i, (k, ya) in enumerate(arrs.items()):
        pts = " ".join(f"{ax.x(a):.1f},{ax.y(b):.1f}" for a, b in zip(xa, ya) if math.isfinite(b))
        body.append(f'<polyline points="{pts}" fill="none" stroke="{_COLORS[i % len(_COLORS)]}" stroke-width="1.5"/>')
        if k:
            body.append(f'<text x="{_W - _PAD}" y="{_PAD + 14 * i}" text-anchor="end" font-size="11" '
                        f'fill="{_COLORS[i % len(_COLORS)]}">{html.escape(k)}</text>')
    return _svg(body, title)


def scatter(x, y, title: str = "", xlabel: str = "", ylabel: str = "", max_points: int = 5000) -> str:
    xa, ya = _arr(x), _arr(y)
    if len(xa) > max_points:  # deterministic thinning keeps the document small
        idx = np.linspace(0, len(xa) - 1, max_points).astype(int)
        xa, ya = xa[idx], ya[idx]
    ax = _Axes(xa.min(), xa.max(), ya.min(), ya.max())
    body = ax.frame(xlabel, ylabel)
    body += [f'<circle cx="{ax.x(a):.1f}" cy="{ax.y(b):.1f}" r="2" fill="{_COLORS[0]}" fill-opacity="0.6"/>'
             for a, b in zip(xa, ya)]
    return _svg(body, title)


def _color(t: float) -> str:
    """t in [0,1] -> blue-white-red."""
    t = min(1.0, max(0.0, t))
    if t < 0.5:
        u = t * 2
        r, g, b = int(255 * u), int(255 * u), 255
    else:
        u = (t - 0.5) * 2
        r, g, b = 255, int(255 * (1 - u)), int(255 * (1 - u))
    return f"#{r:02x}{g:02x}{b:02x}"


def heatmap(matrix, labels=None, title: str = "", vmin=None, vmax=None, annotate: bool = True) -> str:
    m = np.asarray(matrix.detach().cpu() if hasattr(matrix, "detach") else matrix, dtype=np.float64)
    rows, cols = m.shape
    lo = np.nanmin(m) if vmin is None else vmin
    hi = np.nanmax(m) if vmax is None else vmax
    cell = max(12, min(48, (min(_W, _H) - 2 * _PAD) // max(rows, cols)))
    w, h = 2 * _PAD + cols * cell + 80, 2 * _PAD + rows * cell
    body = []
    for i in range(rows):
        for j in range(cols):
            v = m[i, j]
            t = 0.5 if hi == lo or not math.isfinite(v) else (v - lo) / (hi - lo)
            x, y = _PAD + 60 + j * cell, _PAD + i * cell
            body.append(f'<rect x="{x}" y="{y}" width="{cell}" height="{cell}" fill="{_color(t)}"/>')
            if annotate and cell >= 28:
                body.append(f'<text x="{x + cell / 2}" y="{y + cell / 2 + 4}" text-anchor="middle" '
                            f'font-size="9">{_nice(v)}</text>')
    if labels is not None:
        for i, lab in enumerate(labels[:rows]):
            body.append(f'<text x="{_PAD + 56}" y="{_PAD + i * cell + cell / 2 + 4}" text-anchor="end" '
                        f'font-size="10">{html.escape(str(lab))[:14]}</text>')
    return _svg(body, title, w, h)


def geo_heatmap(lat, lon, bins: int = 40, title: str = "", weights=None) -> str:
    """Point density on a lat/lon grid (folium HeatMap): counts binned, drawn as a heatmap."""
    la, lo = _arr(lat), _arr(lon)
    wts = None if weights is None else _arr(weights)
    h, _, _ = np.histogram2d(la, lo, bins=bins, weights=wts)
    return heatmap(h[::-1], title=title, annotate=False)


def save(svg: str, path) -> str:
    """Write an SVG; relative paths resolve inside the project (like hdfs paths)."""
    p = Path(path)
    if not p.is_absolute():
        from . import hdfs

        p = Path(hdfs.abs_path(str(path)))
    p.parent.mkdir(parents=True, exist_ok=True)
    p.write_text(svg)
    return str(p)
