#!/usr/bin/env python3
"""FETCH_SIZE calibration (tools/ubench_fetch_cal.hip under rocprofv3 --pmc
FETCH_SIZE): reported KiB per dispatch against the bytes each kernel moves.
usage: python3 tools/fetch_cal.py OUTDIR > profiles/<tag>_fetch_calibration.txt"""
import csv
import glob
import statistics
import sys

f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == "FETCH_SIZE"]
rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0)))
GIB, READS = 1 << 30, 4_000_000
by = {}
rand_i = 0
for r in rows:
    k, kib = r["Kernel_Name"], float(r["Counter_Value"])
    if "stream16" in k:
        by.setdefault("stream16 (1 GiB, 16 B/lane nt)", []).append(kib * 1024 / GIB)
    elif "stream8" in k:
        by.setdefault("stream8 (1 GiB, 8 B/lane nt)", []).append(kib * 1024 / GIB)
    elif "rand8" in k:
        t = ["8 GiB", "40 MB", "640 KB"][rand_i % 3]
        rand_i += 1
        by.setdefault(f"rand8 table {t} (B reported per random 8-B read)", []).append(kib * 1024 / READS)
print("FETCH_SIZE calibration on gfx950 (tools/ubench_fetch_cal.hip), per dispatch:")
for k, v in by.items():
    unit = "reported / moved bytes" if "stream" in k else "bytes"
    print(f"  {k:56s} median {statistics.median(v):8.3f} {unit}  (dispatches {len(v)}: {', '.join(f'{x:.3f}' for x in v)})")
