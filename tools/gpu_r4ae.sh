#!/bin/bash
# Round 4 GPU call AE: up to 32 pending groups per flush (raw32) against 8
# (raw8) and the committed library -- raw parity on raw32, bench --raw
# interleaved.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
ABNN_LIB=$PWD/tools/exp/raw32.so t 900 python -u -m pytest tests/test_gpu_raw.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/rae_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/rae_tests.log; exit 1; }
tail -2 gpurun_out/rae_tests.log
for r in 1 2; do
  for lib in tools/exp/final_c.so tools/exp/raw8.so tools/exp/raw32.so; do
    ABNN_LIB=$PWD/$lib t 300 python -u bench.py --raw --steps 50 > gpurun_out/br.json 2> gpurun_out/br.err || { echo "raw bench failed"; tail -5 gpurun_out/br.err; exit 1; }
    python3 tools/bench_line.py gpurun_out/br.json "raw $lib r$r"
  done
done | tee gpurun_out/raw_ab_ae.txt
