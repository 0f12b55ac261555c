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


# ------------------------------------------------------------------ maps (folium / ipyleaflet)
# notebooks/ml/Plotting/folium_heat_map.ipynb:37-111 (HeatMapWithTime over moving points) and
# ipyleaflet.ipynb:21-251 (Map, layers, DrawControl with draw callbacks, two maps linked on
# center/zoom).  No tile server or browser widget exists here: a map is a Web-Mercator canvas whose
# layers render to SVG; drawing is an API call that fires the same callbacks with GeoJSON.
def _mercator(lat, lon, center, zoom, w, h):
    """(x, y) pixels of lat/lon for a Web-Mercator view of ``zoom`` centred on ``center``."""
    def proj(la, lo):
        s = 256 * 2 ** zoom
        x = (lo + 180.0) / 360.0 * s
        r = np.radians(np.clip(la, -85.05, 85.05))
        y = (1 - np.log(np.tan(r) + 1 / np.cos(r)) / np.pi) / 2 * s
        return x, y

    cx, cy = proj(np.asarray(center[0], float), np.asarray(center[1], float))
    x, y = proj(np.asarray(lat, float), np.asarray(lon, float))
    return x - cx + w / 2, y - cy + h / 2


class GeoJSON:
    def __init__(self, data: dict, style: dict | None = None):
        self.data, self.style = data, dict(style or {})


class Marker:
    def __init__(self, location, title: str = ""):
        self.location, self.title = tuple(location), title


class Polyline:
    def __init__(self, locations, color: str = "#0000FF"):
        self.locations, self.color = [tuple(p) for p in locations], color


class Polygon(Polyline):
    pass


class Circle:
    def __init__(self, location, radius: float = 1000.0, color: str = "#0000FF"):
        self.location, self.radius, self.color = tuple(location), float(radius), color


class GeoMap:
    """An ipyleaflet ``Map`` / folium ``Map`` stand-in: ``center``, ``zoom``, ``add_layer``,
    ``add_control``, ``to_svg`` / ``save``."""

    def __init__(self, center=(0.0, 0.0), zoom: int = 5, width: int = 640, height: int = 400, layout=None):
        self.center, self.zoom = tuple(center), int(zoom)
        self.width, self.height = width, height
        if layout:
            self.width = int(str(layout.get("width", width)).rstrip("px"))
            self.height = int(str(layout.get("height", height)).rstrip("px"))
        self.layers: list = []
        self.controls: list = []
        self._links: list = []

    def __setattr__(self, k, v):
        object.__setattr__(self, k, v)
        if k in ("center", "zoom"):
            for other, attr in getattr(self, "_links", []):
                if attr == k and getattr(other, k) != v:
                    setattr(other, k, v)

    def add_layer(self, layer):
        self.layers.append(layer)
        return self

    def add_control(self, control):
        self.controls.append(control)
        control.map = self
        return self

    def _xy(self, lat, lon):
        return _mercator(lat, lon, self.center, self.zoom, self.width, self.height)

    def _geojson_svg(self, geom: dict, color: str) -> list[str]:
        t, c = geom.get("type"), geom.get("coordinates")
        out = []
        if t == "Point":
            x, y = self._xy(c[1], c[0])
            out.append(f'<circle cx="{x:.1f}" cy="{y:.1f}" r="5" fill="{color}"/>')
        elif t in ("LineString", "Polygon"):
            ring = c[0] if t == "Polygon" else c
            xs, ys = self._xy([p[1] for p in ring], [p[0] for p in ring])
            pts = " ".join(f"{a:.1f},{b:.1f}" for a, b in zip(xs, ys))
            tag = "polygon" if t == "Polygon" else "polyline"
            out.append(f'<{tag} points="{pts}" fill="{color if t == "Polygon" else "none"}" fill-opacity="0.3" '
                       f'stroke="{color}" stroke-width="2"/>')
        elif t == "Feature":
            out += self._geojson_svg(geom["geometry"], color)
        elif t == "FeatureCollection":
            for f in geom["features"]:
                out += self._geojson_svg(f, color)
        return out

    def to_svg(self, title: str = "") -> str:
        body = [f'<rect width="{self.width}" height="{self.height}" fill="#e8eef2"/>']
        for L in self.layers:
            if isinstance(L, Marker):
                x, y = self._xy(L.location[0], L.location[1])
                body.append(f'<circle cx="{x:.1f}" cy="{y:.1f}" r="6" fill="#d62728"/>')
            elif isinstance(L, Polyline):
                xs, ys = self._xy([p[0] for p in L.locations], [p[1] for p in L.locations])
                pts = " ".join(f"{a:.1f},{b:.1f}" for a, b in zip(xs, ys))
                tag = "polygon" if isinstance(L, Polygon) else "polyline"
                body.append(f'<{tag} points="{pts}" fill="{L.color if tag == "polygon" else "none"}" '
                            f'fill-opacity="0.3" stroke="{L.color}" stroke-width="2"/>')
            elif isinstance(L, Circle):
                x, y = self._xy(L.location[0], L.location[1])
                m_per_px = 156543.03 * np.cos(np.radians(L.location[0])) / 2 ** self.zoom
                body.append(f'<circle cx="{x:.1f}" cy="{y:.1f}" r="{L.radius / m_per_px:.1f}" fill="{L.color}" '
                            'fill-opacity="0.3"/>')
            elif isinstance(L, GeoJSON):
                body += self._geojson_svg(L.data, L.style.get("color", "#0000FF"))
            elif isinstance(L, HeatMapWithTime):
                body += L._frame_svg(self, L.current)
        return _svg(body, title, self.width, self.height)

    def save(self, path, title: str = "") -> str:
        return save(self.to_svg(title), path)


Map = GeoMap


def link(a: tuple, b: tuple):
    """traitlets.link((m, 'center'), (m2, 'center')): the two attributes stay equal."""
    (oa, attr), (ob, attr2) = a, b
    if attr != attr2:
        raise ValueError("link the same attribute of two maps")
    setattr(ob, attr, getattr(oa, attr))
    oa._links.append((ob, attr))
    ob._links.append((oa, attr))
    return (oa, ob, attr)


class DrawControl:
    """ipyleaflet ``DrawControl``: enabled shape tools, ``on_draw`` callbacks receiving
    (control, action, geo_json), ``last_action`` / ``last_draw``, ``clear_*``.  Shapes are drawn
    with :meth:`draw` (the programmatic counterpart of a mouse gesture)."""

    _KIND = {"marker": "Point", "polyline": "LineString", "polygon": "Polygon", "rectangle": "Polygon",
             "circle": "Point", "circlemarker": "Point"}

    def __init__(self, **tools):
        self.tools = {k: v for k, v in tools.items() if k in self._KIND}
        self._handlers: list = []
        self.shapes: list[dict] = []
        self.last_action, self.last_draw = "", {"type": "Feature", "geometry": None}
        self.map = None

    def on_draw(self, fn):
        self._handlers.append(fn)

    def draw(self, kind: str, coordinates, **properties) -> dict:
        if kind not in self.tools:
            raise ValueError(f"draw tool {kind!r} is not enabled on this control")
        if kind == "rectangle":
            (la0, lo0), (la1, lo1) = coordinates
            coordinates = [[[lo0, la0], [lo1, la0], [lo1, la1], [lo0, la1], [lo0, la0]]]
        elif kind in ("marker", "circle", "circlemarker"):
            coordinates = [coordinates[1], coordinates[0]]
        elif kind == "polygon":
            coordinates = [[[lo, la] for la, lo in coordinates] + [[coordinates[0][1], coordinates[0][0]]]]
        elif kind == "polyline":
            coordinates = [[lo, la] for la, lo in coordinates]
        feat = {"type": "Feature", "properties": {"style": self.tools[kind].get("shapeOptions", {}), "kind": kind,
                                                  **properties},
                "geometry": {"type": self._KIND[kind], "coordinates": coordinates}}
        self.shapes.append(feat)
        self.last_action, self.last_draw = "created", feat
        for fn in self._handlers:
            fn(self, "created", feat)
        return feat

    def _clear(self, kinds):
        self.shapes = [s for s in self.shapes if s["properties"]["kind"] not in kinds]
        self.last_action = "deleted"

    def clear_circles(self):
        self._clear({"circle", "circlemarker"})

    def clear_polylines(self):
        self._clear({"polyline"})

    def clear_rectangles(self):
        self._clear({"rectangle"})

    def clear_markers(self):
        self._clear({"marker"})

    def clear_polygons(self):
        self._clear({"polygon"})

    def clear(self):
        self.shapes = []
        self.last_action = "deleted"


class HeatMapWithTime:
    """folium ``plugins.HeatMapWithTime(data, index=None)``: one point-density frame per time step;
    ``data[t]`` is a list of [lat, lon(, weight)].  ``frames(map)`` renders every step, ``current``
    selects the step a map shows (the player slider)."""

    def __init__(self, data, index=None, auto_play: bool = False, max_opacity: float = 0.6, min_speed: float = 0.1,
                 radius: float = 12.0):
        self.data = [np.asarray(t, dtype=np.float64).reshape(len(t), -1) for t in data]
        self.index = list(index) if index is not None else list(range(len(self.data)))
        if len(self.index) != len(self.data):
            raise ValueError("index must have one entry per time step")
        self.max_opacity, self.radius, self.current = float(max_opacity), float(radius), 0

    def add_to(self, m: GeoMap):
        m.add_layer(self)
        return self

    def _frame_svg(self, m: GeoMap, t: int) -> list[str]:
        pts = self.data[t]
        if not len(pts):
            return []
        w = pts[:, 2] if pts.shape[1] > 2 else np.ones(len(pts))
        xs, ys = m._xy(pts[:, 0], pts[:, 1])
        wmax = float(w.max()) or 1.0
        return [f'<circle cx="{x:.1f}" cy="{y:.1f}" r="{self.radius}" fill="{_color(float(v) / wmax)}" '
                f'fill-opacity="{self.max_opacity * 0.5:.2f}"/>' for x, y, v in zip(xs, ys, w)]

    def frames(self, m: GeoMap) -> list[str]:
        out = []
        for t in range(len(self.data)):
            self.current = t
            out.append(m.to_svg(title=str(self.index[t])))
        self.current = 0
        return out

    def centroids(self) -> np.ndarray:
        """Weighted (lat, lon) centre of mass per time step — how the cloud moves."""
        return np.array([np.average(d[:, :2], axis=0, weights=d[:, 2] if d.shape[1] > 2 else None)
                         for d in self.data])
