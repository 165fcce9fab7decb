#!/bin/bash
# Round 4 GPU call Y: where a config-3 pass with plasticity goes now (device
# structural update, partition jump): rocprofv3 kernel trace of bench
# --plasticity.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/y
t() { timeout -k 10 "$@"; }
t 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/y/c3p -o run -- python3 bench.py --plasticity --steps 200 --no-cpu-baseline > gpurun_out/y/c3p.json 2> gpurun_out/y/c3p.err || { echo "prof failed"; tail -5 gpurun_out/y/c3p.err; exit 1; }
python3 tools/bench_line.py gpurun_out/y/c3p.json c3p
cut -d, -f1-7 gpurun_out/y/c3p/run_kernel_stats.csv | head -24
