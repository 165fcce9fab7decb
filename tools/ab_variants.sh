#!/bin/bash
# A/B timing of kernel variants on one box: the in-tree library and every
# tools/exp/*.so (built here with tools/build_variant.sh), interleaved over
# ROUNDS rounds of bench.py.  usage (on the GPU box): tools/ab_variants.sh [ROUNDS] [extra bench args]
set -o pipefail
ROUNDS=${1:-3}
shift
libs=("abnn_amd/libabnn_hip.so" tools/exp/*.so)
mkdir -p gpurun_out
for r in $(seq 1 "$ROUNDS"); do
  for lib in "${libs[@]}"; do
    [ -f "$lib" ] || continue
    n=$(basename "$lib" .so)
    ABNN_LIB=$PWD/$lib timeout -k 10 120 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/ab_${n}_$r.txt 2>&1 || exit 1
    python3 - "$n" "$r" "gpurun_out/ab_${n}_$r.txt" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[3]) if l.startswith("{")][-1])
rf = d["roofline"]
print(f"{sys.argv[1]:>24s} r{sys.argv[2]}  pass {d['ms_per_step']*1e3:6.1f} us  launch avg {rf['avg_launch_ms']*1e3:6.1f} "
      f"median {rf['median_launch_ms']*1e3:6.1f} min {rf['min_launch_ms']*1e3:6.1f}  spikes {d['config']['spikes_per_pass']}")
PY
  done
done
