#!/bin/bash
# Round 4 GPU call A: the whole -m gpu suite on the in-tree library, then the
# reference-layout bench and the c3 plasticity bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
(while sleep 50; do date +%s >> gpurun_out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
t() { timeout -k 10 "$@"; }
t 800 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4a_tests.log; exit 1; }
tail -3 gpurun_out/r4a_tests.log
t 200 python -u bench.py --raw --steps 50 > gpurun_out/bench_raw.json 2> gpurun_out/bench_raw.err || { echo "raw bench failed"; tail -20 gpurun_out/bench_raw.err; exit 1; }
cat gpurun_out/bench_raw.json
t 200 python -u bench.py --plasticity --steps 100 --no-cpu-baseline > gpurun_out/bench_c3p.json 2> gpurun_out/bench_c3p.err || { echo "c3p bench failed"; tail -20 gpurun_out/bench_c3p.err; exit 1; }
head -c 600 gpurun_out/bench_c3p.json
