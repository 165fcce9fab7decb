#!/bin/bash
# Bench every compiled gate shape (ABNN_GATE) once; one process each.
for s in ${SHAPES:-256x8 256x16 512x4 512x8 1024x4}; do
  ABNN_GATE=$s timeout -k 10 240 python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-8} --no-cpu-baseline > gpurun_out/sweep_$s.json 2> gpurun_out/sweep_$s.err
  rc=$?
  python - "$s" <<'PY'
import json, sys
s = sys.argv[1]
try:
    d = json.loads(open(f"gpurun_out/sweep_{s}.json").read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f"{s:8s} {d['value']/1e9:8.2f} Gev/s  pass {d['ms_per_step']:.4f} ms  gate {r['avg_launch_ms']:.4f} ms  frac {r['frac']:.3f}")
except Exception as e:
    print(s, "FAILED", e)
PY
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FATAL rc=$rc at $s"; exit 100; fi
done
