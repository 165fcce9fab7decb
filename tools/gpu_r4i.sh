#!/bin/bash
# Round 4 GPU call I: stamping workgroups' wave 1 walks wave 0's range
# (delegate) -- fused-pass parity tests, then interleaved A/B vs HEAD and
# the wave timelines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
t 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_engine.py tests/test_cpp_api.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r4i_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4i_tests.log; exit 1; }
tail -2 gpurun_out/r4i_tests.log
ROUNDS=4 t 500 bash tools/ab_cfg.sh head=tools/exp/head.so delegate=tools/exp/delegate.so > /dev/null || { echo "ab failed"; exit 1; }
cat gpurun_out/ab_cfg.txt
ABNN_LIB=$PWD/tools/exp/delegate.so t 200 python3 tools/wc_multi.py 200 > gpurun_out/wcm_delegate.txt 2>&1 || echo "wcm failed"
