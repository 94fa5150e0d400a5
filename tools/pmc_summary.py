"""Per-dispatch SQ counters of the last dispatch of a kernel, from
tools/pmc_sq.sh output:  python tools/pmc_summary.py OUTDIR kernel_substring"""
import collections
import csv
import glob
import os
import sys

d, name = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(float)
for sub in ("pmca", "pmcb"):
    for f in glob.glob(os.path.join(d, sub, "*counter_collection.csv")):
        rows = [r for r in csv.DictReader(open(f)) if name in r["Kernel_Name"]]
        if not rows:
            continue
        last = max(int(r["Dispatch_Id"]) for r in rows)
        for r in rows:
            if int(r["Dispatch_Id"]) == last:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
        print(sub, rows[0]["Kernel_Name"][:90], "VGPR", rows[0].get("VGPR_Count"), "SGPR", rows[0].get("SGPR_Count"))
w = acc.get("SQ_WAVES", 0) or 1
for k in sorted(acc):
    print(f"{k:24s} {acc[k]:16.4g}  per wave {acc[k] / w:12.4g}")
