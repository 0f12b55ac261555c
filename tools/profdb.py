"""Summarise a rocprofv3 results.db (kernel-dispatch table): per-kernel totals and one step's timeline.
usage: python tools/profdb.py <run_results.db> [title] [timeline-anchor-kernel-prefix]"""
import sqlite3
import sys

db = sys.argv[1]
title = sys.argv[2] if len(sys.argv) > 2 else db
anchor = sys.argv[3] if len(sys.argv) > 3 else None
c = sqlite3.connect(db)
print(f"# {title}")
print(f"{'calls':>7} {'total_ms':>9} {'avg_us':>8} {'min_us':>8} {'max_us':>8}  kernel")
q = ("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) from kernels "
     "group by name order by sum(end-start) desc limit 30")
for n, k, s, a, mi, ma in c.execute(q):
    print(f"{k:7d} {s / 1e6:9.3f} {a / 1e3:8.2f} {mi / 1e3:8.2f} {ma / 1e3:8.2f}  {n[:110]}")
if anchor:
    rows = list(c.execute("select name, start, end from kernels order by start"))
    idx = [i for i, r in enumerate(rows) if r[0].startswith(anchor)]
    if len(idx) > 20:
        i = idx[len(idx) // 2]
        t0 = rows[i][1]
        print(f"\n# timeline of consecutive dispatches from a mid-run '{anchor}' (us from its start)")
        for r in rows[i:i + 24]:
            print(f"{(r[1] - t0) / 1e3:9.2f} {(r[2] - t0) / 1e3:9.2f}  {r[0][:80]}")
