"""Document index for the Elasticsearch examples (notebooks/spark/Elasticsearch-python.ipynb:66-125:
``hops.elasticsearch.get_elasticsearch_config(index)`` feeding the ES-Spark connector, write a
DataFrame, read it back with a query).

There is no Elasticsearch service in this environment, so indices are local JSONL
documents under ``Elasticsearch/<index>/`` with a small query engine: ``match`` (token
containment), ``term`` (equality), ``range`` (gt/gte/lt/lte), ``bool`` (must/should/
must_not/filter), ``match_all``.  ``write``/``read`` take and return pandas DataFrames.
"""
from __future__ import annotations

import json
import re
from pathlib import Path

import pandas as pd

from . import hdfs


def _dir(index: str) -> Path:
    d = Path(hdfs.project_path()) / "Elasticsearch" / index.lower()
    d.mkdir(parents=True, exist_ok=True)
    return d


def get_elasticsearch_config(index: str) -> dict:
    return {"es.nodes": "127.0.0.1", "es.port": "9200", "es.nodes.wan.only": "true",
            "es.resource": f"{index.lower()}/_doc", "es.net.ssl": "false", "es.index": index.lower(),
            "hopsx.es.path": str(_dir(index))}


def get_elasticsearch_index(index: str) -> str:
    return index.lower()


def index_documents(index: str, docs, id_field: str | None = None, mode: str = "append") -> int:
    p = _dir(index) / "docs.jsonl"
    existing = {} if mode == "overwrite" or not p.exists() else {
        d["_id"]: d for d in (json.loads(l) for l in p.read_text().splitlines() if l)}
    n = len(existing)
    for d in docs:
        d = dict(d)
        _id = str(d[id_field]) if id_field else str(n)
        n += 1
        existing[_id] = {"_id": _id, "_source": d}
    p.write_text("".join(json.dumps(v, default=str) + "\n" for v in existing.values()))
    return len(existing)


def write(df: pd.DataFrame, index: str, id_field: str | None = None, mode: str = "append") -> int:
    return index_documents(index, df.to_dict("records"), id_field, mode)


def _tokens(s) -> set:
    return set(re.findall(r"\w+", str(s).lower()))


def _match(src: dict, q: dict) -> bool:
    if not q or "match_all" in q:
        return True
    if "match" in q:
        (f, v), = q["match"].items()
        v = v["query"] if isinstance(v, dict) else v
        return bool(_tokens(v) & _tokens(src.get(f, "")))
    if "term" in q:
        (f, v), = q["term"].items()
        v = v["value"] if isinstance(v, dict) else v
        return src.get(f) == v
    if "range" in q:
        (f, c), = q["range"].items()
        x = src.get(f)
        if x is None:
            return False
        ops = {"gt": lambda a, b: a > b, "gte": lambda a, b: a >= b, "lt": lambda a, b: a < b,
               "lte": lambda a, b: a <= b}
        return all(ops[k](x, v) for k, v in c.items())
    if "bool" in q:
        b = q["bool"]
        must = b.get("must", []) + b.get("filter", [])
        must = must if isinstance(must, list) else [must]
        ok = all(_match(src, m) for m in must)
        should = b.get("should", [])
        should = should if isinstance(should, list) else [should]
        if should:
            ok = ok and any(_match(src, m) for m in should)
        mn = b.get("must_not", [])
        mn = mn if isinstance(mn, list) else [mn]
        return ok and not any(_match(src, m) for m in mn)
    raise ValueError(f"unsupported query {q}")


def search(index: str, query: dict | None = None, size: int = 10_000) -> dict:
    p = _dir(index) / "docs.jsonl"
    docs = [json.loads(l) for l in p.read_text().splitlines() if l] if p.exists() else []
    q = (query or {}).get("query", query or {})
    hits = [d for d in docs if _match(d["_source"], q)][:size]
    return {"hits": {"total": {"value": len(hits)}, "hits": hits}}


def read(index: str, query: dict | None = None) -> pd.DataFrame:
    return pd.DataFrame([h["_source"] for h in search(index, query)["hits"]["hits"]])


def delete_index(index: str) -> None:
    import shutil

    shutil.rmtree(_dir(index), ignore_errors=True)
