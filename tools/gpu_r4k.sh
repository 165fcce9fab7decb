#!/bin/bash
# Round 4 GPU call K: tail issue priority 3 (t3), with the progress-ranked
# stream priority (pp_t3) -- parity on pp_t3, interleaved A/B vs HEAD and
# progprio, wave timelines of both new variants.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/wck_pp_t3 gpurun_out/wck_t3
t() { timeout -k 10 "$@"; }
ABNN_LIB=$PWD/tools/exp/pp_t3.so t 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4k_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4k_tests.log; exit 1; }
tail -2 gpurun_out/r4k_tests.log
ROUNDS=3 t 700 bash tools/ab_cfg.sh head=tools/exp/head.so t3=tools/exp/t3.so pp_t3=tools/exp/pp_t3.so progprio=tools/exp/progprio.so > /dev/null || { echo "ab failed"; exit 1; }
cat gpurun_out/ab_cfg.txt
ABNN_LIB=$PWD/tools/exp/pp_t3.so OUT=gpurun_out/wck_pp_t3 t 200 python3 tools/wc_multi.py 200 > gpurun_out/wcm_pp_t3.txt 2>&1 || echo "wcm failed"
ABNN_LIB=$PWD/tools/exp/t3.so OUT=gpurun_out/wck_t3 t 200 python3 tools/wc_multi.py 200 > gpurun_out/wcm_t3.txt 2>&1 || echo "wcm failed"
tail -3 gpurun_out/wcm_pp_t3.txt gpurun_out/wcm_t3.txt
