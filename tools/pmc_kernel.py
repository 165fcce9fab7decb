#!/usr/bin/env python3
"""Per-launch counter values of one kernel from rocprofv3 --pmc CSVs under a
directory (every *counter_collection.csv found): median over the kernel's
dispatches of each counter.  usage: tools/pmc_kernel.py DIR KERNEL"""
import csv
import glob
import statistics
import sys

d, kern = sys.argv[1], sys.argv[2]
vals = {}
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    per = {}
    for r in csv.DictReader(open(f)):
        if not r.get("Kernel_Name", "").startswith(kern):
            continue
        key = (r["Counter_Name"], r["Dispatch_Id"])
        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    for (name, _), v in per.items():
        vals.setdefault(name, []).append(v)
for name, v in sorted(vals.items()):
    print(f"{kern} {name}: median {statistics.median(v):.4g} over {len(v)} launches (min {min(v):.4g}, max {max(v):.4g})")
