#!/bin/bash
# Round 4 GPU call U: a full-step partition move when a range costs over 4x
# the mean (jump) -- parity on the variant, then config 3 with plasticity
# (structural updates every 50 passes) and the plain config-3 pass,
# interleaved against the committed library.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
ABNN_LIB=$PWD/tools/exp/jump.so t 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plasticity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4u_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4u_tests.log; exit 1; }
tail -2 gpurun_out/r4u_tests.log
for r in 1 2; do
  for lib in tools/exp/items_c.so tools/exp/jump.so; do
    ABNN_LIB=$PWD/$lib t 300 python -u bench.py --plasticity --steps 200 --no-cpu-baseline > gpurun_out/bp.json 2> gpurun_out/bp.err || { echo "c3p bench failed"; tail -5 gpurun_out/bp.err; exit 1; }
    python3 tools/bench_line.py gpurun_out/bp.json "c3p $lib r$r"
  done
done | tee gpurun_out/c3p_ab_u.txt
ROUNDS=3 t 400 bash tools/ab_cfg.sh base=tools/exp/items_c.so jump=tools/exp/jump.so > /dev/null || { echo "ab failed"; exit 1; }
cat gpurun_out/ab_cfg.txt
