#!/bin/bash
# Round 4 GPU call D: where the reference-layout pass's time goes (rocprofv3
# kernel trace of bench.py --raw), and the fused pass's rocprof trace on the
# current kernel.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
t 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_raw -o run -- python3 bench.py --raw --steps 50 > gpurun_out/bench_raw_prof.json 2> gpurun_out/bench_raw_prof.err || { echo "raw prof failed"; tail -5 gpurun_out/bench_raw_prof.err; exit 1; }
f=$(find gpurun_out/prof_raw -name "*kernel_stats.csv" | head -1); head -20 "$f"
