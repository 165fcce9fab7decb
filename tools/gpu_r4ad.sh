#!/bin/bash
# Round 4 GPU call AD: the reference-layout gate with its refractory rounds
# deferred over up to 8 groups (no per-group pipeline drain) -- raw parity
# (pass by pass, budgets, a pool too small, config 3), then bench --raw
# interleaved against the committed library.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
t 900 python -u -m pytest tests/test_gpu_raw.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/rad_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/rad_tests.log; exit 1; }
tail -2 gpurun_out/rad_tests.log
for r in 1 2; do
  for lib in tools/exp/final_c.so abnn_amd/libabnn_hip.so; do
    ABNN_LIB=$PWD/$lib t 300 python -u bench.py --raw --steps 50 > gpurun_out/br.json 2> gpurun_out/br.err || { echo "raw bench failed"; tail -5 gpurun_out/br.err; exit 1; }
    python3 tools/bench_line.py gpurun_out/br.json "raw $lib r$r"
  done
done | tee gpurun_out/raw_ab_ad.txt
