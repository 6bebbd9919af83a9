"""Summarise a rocprofv3 --pmc counter_collection.csv: per-kernel mean of each counter."""
import collections
import csv
import sys

for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(list)
    meta = {}
    for r in rows:
        k = (r["Kernel_Name"][:60], r["Counter_Name"])
        agg[k].append(float(r["Counter_Value"]))
        meta[r["Kernel_Name"][:60]] = (r.get("VGPR_Count"), r.get("LDS_Block_Size"), r.get("Grid_Size"))
    for (kn, cn), v in sorted(agg.items()):
        print(f"{kn:60s} {cn:28s} n={len(v):3d} mean={sum(v)/len(v):.4g}")
    for kn, m in meta.items():
        print("meta", kn, m)
