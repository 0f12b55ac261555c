"""Side-by-side table of tools/gpu_gg_ab.sh outputs: per layer, glds us of every variant."""
import json
import sys
from pathlib import Path

d = Path(sys.argv[1])
variants = ["default", "diag", "smax2", "smax1", "smax1_diag"]
rows = {}
for v in variants:
    f = d / f"{v}.jsonl"
    if not f.exists():
        continue
    for ln in f.read_text().splitlines():
        if not ln.startswith("{") or '"H"' not in ln:
            continue
        r = json.loads(ln)
        key = (r["H"], r["C"], r["CO"], r["k"], r["s"], r["n"])
        rows.setdefault(key, {})[v] = r.get("glds_us", float("nan"))
print("H C CO k s n | " + " ".join(f"{v:>10}" for v in variants))
tot = {v: 0.0 for v in variants}
for key, vals in rows.items():
    print(" ".join(map(str, key)) + " | " + " ".join(f"{vals.get(v, float('nan')):10.1f}" for v in variants))
    for v in variants:
        tot[v] += vals.get(v, 0.0) * key[5]
print("step total us | " + " ".join(f"{tot[v]:10.1f}" for v in variants))
