#!/bin/bash
# Round 4 GPU call G: the measurement set on this tree -- default bench (c3,
# with the CPU baseline's thread sweep), full sweep, random mode, c3 and c5
# with plasticity, the sharded pass and its all-gather alone at world 1.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
b() { local name=$1; shift; t 400 python -u bench.py "$@" > gpurun_out/g_$name.json 2> gpurun_out/g_$name.err || { echo "bench $name failed"; tail -5 gpurun_out/g_$name.err; exit 1; }; python3 tools/bench_line.py gpurun_out/g_$name.json "$name"; }
b c3 --steps 200
b sweep --events 1000000000 --steps 50 --no-cpu-baseline
b random --mode random --steps 50 --no-cpu-baseline
b c3p --plasticity --steps 100 --no-cpu-baseline
b c5 --config c5 --steps 100 --no-cpu-baseline
b c5p --config c5 --plasticity --steps 100 --no-cpu-baseline
b shard --shard-path --steps 200 --no-cpu-baseline
t 200 python -u tools/allgather_time.py > gpurun_out/allgather.txt 2>&1 || { echo "allgather failed"; tail -5 gpurun_out/allgather.txt; }
cat gpurun_out/allgather.txt
