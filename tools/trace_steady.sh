#!/bin/bash
# Kernel trace of a short bench run and its steady-state per-kernel medians.
# usage: tools/trace_steady.sh TAG [bench args...]   (writes gpurun_out/trace_TAG/)
tag=$1; shift
export TMPDIR=/tmp
out=gpurun_out/trace_$tag
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$out" -o run -- \
    python3 bench.py --steps 30 --warmup 10 --no-cpu-baseline "$@" > "$out/bench.json" 2> "$out/stderr.log"
rc=$?
if [ $rc -ne 0 ]; then echo "FATAL trace rc=$rc"; tail -5 "$out/stderr.log"; exit 100; fi
python3 - "$out" <<'P'
import sys, statistics
sys.path.insert(0, 'tools')
from pmc_summary import steady, find
per, spans = steady(find(sys.argv[1], '*kernel_trace.csv'))
for k, v in per.items():
    print(f"{k:28s} median {statistics.median(v):8.2f}  min {min(v):8.2f}  mean {statistics.mean(v):8.2f}")
print(f"pass span median {statistics.median(spans):.2f} us")
P
tail -c 400 "$out/bench.json"
