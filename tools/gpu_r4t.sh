#!/bin/bash
# Round 4 GPU call T: where a config-3 pass with plasticity goes -- rocprofv3
# kernel stats of bench --plasticity, its wave timelines (tools/wc_multi.py
# with PLASTICITY=1 is not wired: the bench's own per-kernel stats instead).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/t
t() { timeout -k 10 "$@"; }
t 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/t/c3p -o run -- python3 bench.py --plasticity --steps 100 --no-cpu-baseline > gpurun_out/t/c3p.json 2> gpurun_out/t/c3p.err || { echo "prof failed"; tail -5 gpurun_out/t/c3p.err; exit 1; }
python3 tools/bench_line.py gpurun_out/t/c3p.json c3p
cut -d, -f1-7 gpurun_out/t/c3p/run_kernel_stats.csv | head -20
