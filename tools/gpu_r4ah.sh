#!/bin/bash
# Round 4 GPU call AH: the structural update's in-place compaction on
# uploaded tombstone patterns (tests/test_gpu_plasticity.py).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
t 600 python -u -m pytest tests/test_gpu_plasticity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/rah_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/rah_tests.log; exit 1; }
tail -14 gpurun_out/rah_tests.log
