#!/bin/bash
# Round 4 GPU call O: next-bitmap items before the look-back and a shard walk
# that issues every read before its first store (itemsw) -- parity on the
# variant (fused, shard, plasticity), then interleaved A/B against the
# committed library: the fused pass (pass_times) and the sharded pass at
# world 1 (bench --shard-path).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
ABNN_LIB=$PWD/tools/exp/itemsw.so t 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plasticity.py tests/test_sharded_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4o_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4o_tests.log; exit 1; }
tail -2 gpurun_out/r4o_tests.log
ROUNDS=3 t 500 bash tools/ab_cfg.sh base=tools/exp/t3pro_c.so itemsw=tools/exp/itemsw.so > /dev/null || { echo "ab failed"; exit 1; }
cat gpurun_out/ab_cfg.txt
for r in 1 2 3; do
  for lib in tools/exp/t3pro_c.so tools/exp/itemsw.so; do
    ABNN_LIB=$PWD/$lib t 200 python -u bench.py --shard-path --steps 200 --no-cpu-baseline > gpurun_out/bs.json 2> gpurun_out/bs.err || { echo "shard bench failed"; tail -5 gpurun_out/bs.err; exit 1; }
    python3 tools/bench_line.py gpurun_out/bs.json "$lib r$r"
  done
done | tee gpurun_out/shard_ab_o.txt
