#!/bin/bash
# Round 4 GPU call AF: the final evidence on this tree -- whole -m gpu
# suite, rocprofv3 trace + PMC traffic of config 3 (tools/profile.sh), the
# wave timelines and the bench set (driver-shaped default, c3 with the CPU
# baseline, full sweep, random, c3p, c5p, the sharded pass, --raw).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
t 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/raf_suite.log 2>&1 || { echo "suite failed"; tail -40 gpurun_out/raa_suite.log; exit 1; }
tail -2 gpurun_out/raf_suite.log
t 700 bash tools/profile.sh r04af c3 > gpurun_out/prof_r04af.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/prof_r04af.log; exit 1; }
tail -3 gpurun_out/prof_r04af.log
t 200 python3 tools/wc_multi.py 200 > gpurun_out/wcm_r04af.txt 2>&1 || echo "wcm failed"
b() { local name=$1; shift; t 400 python -u bench.py "$@" > gpurun_out/af_$name.json 2> gpurun_out/af_$name.err || { echo "bench $name failed"; tail -5 gpurun_out/af_$name.err; exit 1; }; python3 tools/bench_line.py gpurun_out/af_$name.json "$name"; }
b driver --steps 20 --warmup 5
b c3 --steps 200
b sweep --events 1000000000 --steps 50 --no-cpu-baseline
b random --mode random --steps 50 --no-cpu-baseline
b c3p --plasticity --steps 200 --no-cpu-baseline
b c5p --config c5 --plasticity --steps 100 --no-cpu-baseline
b shard --shard-path --steps 200 --no-cpu-baseline
b raw --raw --steps 100
t 900 bash tools/profile_raw.sh r04af_raw > gpurun_out/prof_r04af_raw.log 2>&1 || { echo "raw profile failed"; tail -20 gpurun_out/prof_r04af_raw.log; exit 1; }
