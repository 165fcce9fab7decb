#!/bin/bash
# Round 4, first GPU call: the raw launcher's tests and bench, the structural
# update's tests (plasticity suite, c5 full size), bench with plasticity, then
# the SQ counters of the unchanged fused pass and the CPU baseline's scaling.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
(while sleep 50; do date +%s >> gpurun_out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
t() { timeout -k 10 "$@"; }
t 700 python -u -m pytest tests/test_gpu_raw.py tests/test_cpp_api.py tests/test_gpu_plasticity.py tests/test_sharded_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4a_tests.log; exit 1; }
tail -3 gpurun_out/r4a_tests.log
t 300 python -u bench.py --raw --steps 50 > gpurun_out/bench_raw.json 2> gpurun_out/bench_raw.err || { echo "raw bench failed"; tail -20 gpurun_out/bench_raw.err; exit 1; }
cat gpurun_out/bench_raw.json
t 400 python -u bench.py --plasticity --steps 100 --no-cpu-baseline > gpurun_out/bench_c3p.json 2> gpurun_out/bench_c3p.err || { echo "c3p bench failed"; tail -20 gpurun_out/bench_c3p.err; exit 1; }
t 900 python -u -m pytest tests/test_gpu_scale.py -k c5 -m gpu -x -v --timeout 850 --timeout-method thread > gpurun_out/r4a_c5.log 2>&1 || { echo "c5 test failed"; tail -40 gpurun_out/r4a_c5.log; exit 1; }
tail -3 gpurun_out/r4a_c5.log
ROUNDS=3 t 600 bash tools/ab_cfg.sh base=tools/exp/base.so noknobs=. > /dev/null || { echo "ab failed"; exit 1; }
cat gpurun_out/ab_cfg.txt
ABNN_LIB=$PWD/tools/exp/base.so t 400 tools/sq_profile.sh gpurun_out/sq_base.txt > /dev/null || { echo "sq base failed"; exit 1; }
t 400 tools/sq_profile.sh gpurun_out/sq_noknobs.txt > /dev/null || { echo "sq new failed"; exit 1; }
t 300 python3 tools/cpu_scaling.py 3 16 64 all > gpurun_out/cpu_scaling.txt 2>&1 || echo "cpu scaling failed"
