#!/bin/bash
# Round 4 GPU call H: the committed evidence for the default bench -- the
# rocprofv3 trace and PMC traffic of config 3 (tools/profile.sh), the wave
# timelines, then a driver-shaped default bench run (--steps 20 --warmup 5).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
t 900 bash tools/profile.sh r04h c3 > gpurun_out/prof_r04h.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/prof_r04h.log; exit 1; }
tail -5 gpurun_out/prof_r04h.log
t 200 python3 tools/wc_multi.py 200 > gpurun_out/wcm_r04h.txt 2>&1 || echo "wcm failed"
t 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver_shape.json 2> gpurun_out/bench_driver_shape.err || { echo "bench failed"; tail -5 gpurun_out/bench_driver_shape.err; exit 1; }
python3 tools/bench_line.py gpurun_out/bench_driver_shape.json "driver-shaped"
