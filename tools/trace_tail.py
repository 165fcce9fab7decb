#!/usr/bin/env python3
"""Per-kernel medians over the last N passes of a kernel-trace CSV, whatever
kernels a pass launches (a pass starts at each k_gate; its span runs to the
next k_gate's start).  usage: python tools/trace_tail.py TRACE_DIR [passes]"""
import collections
import glob
import os
import statistics
import sys
import csv

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
ks = [(r["Kernel_Name"].split("(")[0].split("<")[0].split(" ")[-1], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
      for r in rows if not r["Kernel_Name"].startswith("__amd")]
starts = [i for i, k in enumerate(ks) if k[0].endswith("k_gate")]
passes = list(zip(starts[:-1], starts[1:]))[-n:]
per = collections.defaultdict(list)
spans = []
for a, b in passes:
    spans.append((ks[b][1] - ks[a][1]) / 1000)
    for k in ks[a:b]:
        per[k[0]].append((k[2] - k[1]) / 1000)
    # kernels launched before the gate of the same pass (k_bitmap) belong to it
for k, v in per.items():
    print(f"{k:28s} median {statistics.median(v):8.2f}  min {min(v):8.2f}  launches/pass {len(v) / len(passes):.2f}")
print(f"pass span (gate to gate) median {statistics.median(spans):.2f} us over {len(passes)} passes")
