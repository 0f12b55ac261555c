"""Per-kernel PMC counter sums from rocprofv3 --pmc result databases.
usage: python tools/pmcdb.py <run_results.db> [...] [--match SUBSTR]"""
import sqlite3
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = ""
if "--match" in sys.argv:
    match = sys.argv[sys.argv.index("--match") + 1]
    args = [a for a in args if a != match]
for db in args:
    c = sqlite3.connect(db)
    q = ("select kernel_name, counter_name, sum(value), count(distinct dispatch_id), avg(duration) from counters_collection "
         "where kernel_name like ? group by kernel_name, counter_name order by kernel_name, counter_name")
    cur = None
    for k, n, v, d, dur in c.execute(q, (f"%{match}%",)):
        if k != cur:
            cur = k
            print(f"# {k[:120]}  dispatches={d} avg_dur_us={dur / 1e3:.1f}")
        print(f"  {n:32s} {v / d:16.1f} per dispatch")
