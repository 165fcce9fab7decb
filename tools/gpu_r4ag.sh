#!/bin/bash
# Round 4 GPU call AG: the driver's round-end steps on this tree -- smoke()
# and the default bench with no flags.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
t 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
t 400 python -u bench.py > gpurun_out/default_bench.json 2> gpurun_out/default_bench.err || { echo "bench failed"; tail -5 gpurun_out/default_bench.err; exit 1; }
python3 tools/bench_line.py gpurun_out/default_bench.json default
