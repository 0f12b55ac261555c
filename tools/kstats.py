"""Print a rocprofv3 kernel_stats.csv as a short table (name, calls, avg us, %)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = 0.0
for x in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    print(f"{x['Name'][:64]:64s} {x['Calls']:>6} {float(x['AverageNs']) / 1000:8.2f} us {float(x['Percentage']):6.2f}%")
