#!/bin/bash
# Round 4 GPU call J: issue priority ranked by progress among a SIMD's waves
# (progprio) -- fused-pass parity on the variant, interleaved A/B vs HEAD,
# and the variant's wave timelines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/wcj
t() { timeout -k 10 "$@"; }
ABNN_LIB=$PWD/tools/exp/progprio.so t 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4j_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4j_tests.log; exit 1; }
tail -2 gpurun_out/r4j_tests.log
ROUNDS=4 t 500 bash tools/ab_cfg.sh head=tools/exp/head.so progprio=tools/exp/progprio.so > /dev/null || { echo "ab failed"; exit 1; }
cat gpurun_out/ab_cfg.txt
ABNN_LIB=$PWD/tools/exp/progprio.so OUT=gpurun_out/wcj t 200 python3 tools/wc_multi.py 200 > gpurun_out/wcm_progprio.txt 2>&1 || echo "wcm failed"
cat gpurun_out/wcm_progprio.txt
