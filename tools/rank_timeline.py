"""Interleave the kernel traces of several ranks (tools/rehearse_prof.sh r<k>.db files) on one clock.
usage: python tools/rank_timeline.py <dir> <nranks> [anchor-kernel-prefix] [ndisp]
Prints, per rank, the busy share of the window between the first and the last anchor dispatch, the top
kernels inside it, and the merged timeline of the last ``ndisp`` dispatches (us, rank, duration, kernel)."""
import sqlite3
import sys

d, n = sys.argv[1], int(sys.argv[2])
anchor = sys.argv[3] if len(sys.argv) > 3 else None
nd = int(sys.argv[4]) if len(sys.argv) > 4 else 60
rows = []
for r in range(n):
    c = sqlite3.connect(f"{d}/r{r}.db")
    rows += [(s, e, r, name) for name, s, e in c.execute("select name, start, end from kernels order by start")]
rows.sort()
if anchor:
    a = [x for x in rows if x[3].startswith(anchor)]
    lo, hi = (a[0][0], a[-1][1]) if a else (rows[0][0], rows[-1][1])
else:
    lo, hi = rows[0][0], rows[-1][1]
win = [x for x in rows if x[0] >= lo and x[1] <= hi]
print(f"# window {(hi - lo) / 1e6:.3f} ms from the first to the last '{anchor}' dispatch")
for r in range(n):
    mine = [x for x in win if x[2] == r]
    busy = sum(x[1] - x[0] for x in mine)
    print(f"rank {r}: {len(mine)} dispatches, kernel time {busy / 1e6:.3f} ms ({100 * busy / max(1, hi - lo):.1f} % of the window)")
    tot = {}
    for s, e, _, name in mine:
        k = name.split("(")[0][:70]
        t = tot.setdefault(k, [0, 0])
        t[0] += 1
        t[1] += e - s
    for k, (c_, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:8]:
        print(f"    {c_:6d} {t / 1e6:9.3f} ms  {k}")
t0 = win[-nd][0] if len(win) >= nd else lo
print(f"\n# last {nd} dispatches of the window (us from the first shown)")
for s, e, r, name in win[-nd:]:
    print(f"{(s - t0) / 1e3:10.2f} r{r} {(e - s) / 1e3:8.2f}  {name[:90]}")
