#!/usr/bin/env python3
"""Relate a pass's per-wave s_memrealtime timeline (100 MHz) to the rocprofv3
kernel trace of the same run: prints the last fused kernel's dispatch
start/end next to the first wave entry and the last recorded event, in the
trace's ns (assumes the trace's timestamps count the same 100 MHz clock, x10).
usage: tools/align_clock.py <trace dir> <wave_clock .npy> <finalizer .npy>"""
import csv, glob, sys
import numpy as np

tr = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(tr)), key=lambda r: int(r["Start_Timestamp"]))
g = [r for r in rows if "k_gate" in r["Kernel_Name"]][-1]
s, e = int(g["Start_Timestamp"]), int(g["End_Timestamp"])
w = np.load(sys.argv[2]).astype(np.int64)
tf = np.load(sys.argv[3]).astype(np.int64)
first_entry = w[:, 3].min() * 10
last = max(w[:, 5].max(), tf[2:].max()) * 10
print(f"kernel {s} .. {e}  ({(e - s) / 1e3:.1f} us)")
print(f"waves  {first_entry} .. {last}  ({(last - first_entry) / 1e3:.1f} us)")
print(f"dispatch -> first entry {(first_entry - s) / 1e3:.1f} us; last event -> kernel end {(e - last) / 1e3:.1f} us")
