"""Host-side timeline around the persistent kernel launches from a rocprofv3 --runtime-trace --kernel-trace
results.db: for each mnist_persist_k dispatch, the HIP API calls in the 200 us before it and the sync after it,
so the launch path's host cost (argument build, memset, hipLaunchKernel, synchronize) can be read off.
usage: python tools/launch_gaps.py <results.db> [kernel-prefix]"""
import sqlite3
import sys

db = sys.argv[1]
pref = sys.argv[2] if len(sys.argv) > 2 else "void mnistp::mnist_persist_k"
c = sqlite3.connect(db)
tables = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
api_t = next((t for t in tables if t.lower() in ("regions", "hip_api", "api")), None)
if api_t is None:
    api_t = next((t for t in tables if "region" in t.lower() or "api" in t.lower()), None)
print("# tables:", ", ".join(tables))
ks = list(c.execute("select name, start, end from kernels order by start"))
kp = [k for k in ks if k[0].startswith(pref)]
cols = [r[1] for r in c.execute(f"pragma table_info({api_t})")] if api_t else []
print("# api table:", api_t, cols)
if not api_t:
    sys.exit(0)
ncol = "name" if "name" in cols else cols[1]
api = list(c.execute(f"select {ncol}, start, end from {api_t} order by start"))
for name, s, e in kp[-4:]:
    print(f"\n# kernel {(e - s) / 1e3:.1f} us; API calls from 300 us before its start to 100 us after its end")
    for an, a0, a1 in api:
        if s - 300e3 <= a0 <= e + 100e3:
            print(f"  {(a0 - s) / 1e3:9.1f} .. {(a1 - s) / 1e3:9.1f} us  {an[:60]}")
