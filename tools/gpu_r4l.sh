#!/bin/bash
# Round 4 GPU call L: the prologue waits for its LDS-DMAs only and the fused
# pass zeroes the next images at its end (t3pro, on top of tail priority 3)
# -- fused/shard/plasticity parity on the variant, interleaved A/B, timelines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/wcl
t() { timeout -k 10 "$@"; }
ABNN_LIB=$PWD/tools/exp/t3pro.so t 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plasticity.py tests/test_sharded_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4l_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4l_tests.log; exit 1; }
tail -2 gpurun_out/r4l_tests.log
ROUNDS=4 t 700 bash tools/ab_cfg.sh head=tools/exp/head.so t3=tools/exp/t3.so t3pro=tools/exp/t3pro.so > /dev/null || { echo "ab failed"; exit 1; }
cat gpurun_out/ab_cfg.txt
ABNN_LIB=$PWD/tools/exp/t3pro.so OUT=gpurun_out/wcl t 200 python3 tools/wc_multi.py 200 > gpurun_out/wcm_t3pro.txt 2>&1 || echo "wcm failed"
cat gpurun_out/wcm_t3pro.txt
