#!/bin/bash
# Round 4 GPU call N: the committed evidence on this tree -- rocprofv3 trace
# and PMC traffic of config 3 (tools/profile.sh), wave timelines, the
# driver-shaped default bench, then the measurement set of call G.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
t 900 bash tools/profile.sh r04n c3 > gpurun_out/prof_r04n.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/prof_r04n.log; exit 1; }
tail -5 gpurun_out/prof_r04n.log
t 200 python3 tools/wc_multi.py 200 > gpurun_out/wcm_r04n.txt 2>&1 || echo "wcm failed"
b() { local name=$1; shift; t 400 python -u bench.py "$@" > gpurun_out/n_$name.json 2> gpurun_out/n_$name.err || { echo "bench $name failed"; tail -5 gpurun_out/n_$name.err; exit 1; }; python3 tools/bench_line.py gpurun_out/n_$name.json "$name"; }
b driver --steps 20 --warmup 5
b c3 --steps 200
b sweep --events 1000000000 --steps 50 --no-cpu-baseline
b c3p --plasticity --steps 100 --no-cpu-baseline
b c5p --config c5 --plasticity --steps 100 --no-cpu-baseline
b shard --shard-path --steps 200 --no-cpu-baseline
