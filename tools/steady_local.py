#!/usr/bin/env python3
"""Steady-state per-kernel medians of a kernel-trace directory (last 30 passes)."""
import statistics
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import steady, find

per, spans = steady(find(sys.argv[1], '*kernel_trace.csv'))
for k, v in per.items():
    print(f"{k:28s} median {statistics.median(v):8.2f}  min {min(v):8.2f}  mean {statistics.mean(v):8.2f}")
print(f"pass span median {statistics.median(spans):.2f} us")
