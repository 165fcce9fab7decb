#!/usr/bin/env python3
"""Print a short summary of the bench JSON line in FILE (the last line that
starts with '{').  usage: python tools/bench_line.py FILE [LABEL]"""
import json
import sys

line = [ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1]
b = json.loads(line)
r = b.get("roofline") or {}
print(f"{sys.argv[2] if len(sys.argv) > 2 else ''} {b['ms_per_step'] * 1e3:.1f} us/pass  {b['value'] / 1e9:.1f} G ev/s  "
      f"gate {r.get('avg_launch_ms', 0) * 1e3:.1f} us  frac {r.get('frac')}")
