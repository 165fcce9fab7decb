#!/bin/bash
# Round 4 GPU call E: raw launcher tests + bench + kernel trace after the
# launch-overhead fixes.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
t 400 python -u -m pytest tests/test_gpu_raw.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4e_raw.log 2>&1 || { echo "raw tests failed"; tail -30 gpurun_out/r4e_raw.log; exit 1; }
tail -2 gpurun_out/r4e_raw.log
t 200 python -u bench.py --raw --steps 50 > gpurun_out/bench_raw.json 2> gpurun_out/bench_raw.err || { echo "raw bench failed"; tail -20 gpurun_out/bench_raw.err; exit 1; }
python3 -c "import json; b=json.load(open('gpurun_out/bench_raw.json')); print('raw', b['ms_per_step'], b['roofline']['avg_launch_ms'], b['roofline']['frac'], b['value']/1e9)"
rm -rf gpurun_out/prof_raw
t 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_raw -o run -- python3 bench.py --raw --steps 50 > gpurun_out/bench_raw_prof.json 2> gpurun_out/bench_raw_prof.err || { echo "raw prof failed"; tail -5 gpurun_out/bench_raw_prof.err; exit 1; }
f=$(find gpurun_out/prof_raw -name "*kernel_stats.csv" | head -1); head -14 "$f"
