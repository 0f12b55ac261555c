"""Print the ordered kernel dispatches of one mid-run training step from a rocprofv3 results.db
(the step = the dispatches between two consecutive optimizer-kernel dispatches), with counts of the
non-hopsx kernels (at::native, copyBuffer, fillBuffer) per step.
usage: python tools/step_kernels.py <results.db> [anchor-prefix (default: the optimizer kernel)]"""
import sqlite3
import sys

db = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "void optim_k"
rows = list(sqlite3.connect(db).execute("select name, start, end from kernels order by start"))
idx = [i for i, r in enumerate(rows) if r[0].startswith(anchor)]
if len(idx) < 3:
    sys.exit(f"fewer than 3 '{anchor}' dispatches")
a, b = idx[len(idx) // 2 - 1], idx[len(idx) // 2]
step = rows[a + 1:b + 1]
print(f"# one step: {len(step)} dispatches, {(step[-1][2] - step[0][1]) / 1e3:.1f} us first start -> last end")
foreign = {}
for n, s, e in step:
    short = n.split("(")[0][:110]
    tag = ""
    if "at::native" in n or "rocclr" in n:
        tag = "  <-- non-hopsx"
        foreign[short] = foreign.get(short, 0) + 1
    print(f"{(s - step[0][1]) / 1e3:9.2f} {(e - s) / 1e3:7.2f}  {short}{tag}")
print("# non-hopsx kernels in the step:", foreign if foreign else "none")
