"""Per-kernel mean counter values per wave from rocprofv3 --pmc csv files: pmcsum.py dir [dir...]"""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    if "at::native" in k or "rocclr" in k or "igemm" in k or "SubTensor" in k:
        continue
    waves = sum(v["SQ_WAVES"]) / len(v["SQ_WAVES"])
    row = {c: round(sum(x) / len(x) / waves, 1) for c, x in v.items() if c != "SQ_WAVES"}
    print(k, "waves", round(waves), row)
