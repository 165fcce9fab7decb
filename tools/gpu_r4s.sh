#!/bin/bash
# Round 4 GPU call S: the shard walk with every read issued first, in one
# round trip (sw2) -- parity on the variant, the sharded pass at world 1
# interleaved against the committed library, both walks' timelines; then the
# partition probe's raw arrays.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/probe
t() { timeout -k 10 "$@"; }
ABNN_LIB=$PWD/tools/exp/sw2.so t 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plasticity.py tests/test_sharded_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4s_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4s_tests.log; exit 1; }
tail -2 gpurun_out/r4s_tests.log
for r in 1 2 3; do
  for lib in tools/exp/items_c.so tools/exp/sw2.so; do
    ABNN_LIB=$PWD/$lib t 200 python -u bench.py --shard-path --steps 200 --no-cpu-baseline > gpurun_out/bs.json 2> gpurun_out/bs.err || { echo "shard bench failed"; tail -5 gpurun_out/bs.err; exit 1; }
    python3 tools/bench_line.py gpurun_out/bs.json "$lib r$r"
  done
done | tee gpurun_out/shard_ab_s.txt
for v in items_c sw2; do
  echo "== $v"; ABNN_LIB=$PWD/tools/exp/$v.so t 200 python3 tools/shard_clock.py 100 2>&1 | grep -v "amdgpu.ids\|RCCL\|HIP version\|ROCm version\|Hostname\|Librccl\|Gloo\|c10d" | tail -8
done
OUT=gpurun_out/probe t 300 python3 tools/partition_probe.py 200 > gpurun_out/probe/partition_probe.txt 2>&1 || { echo "probe failed"; tail -5 gpurun_out/probe/partition_probe.txt; exit 1; }
cat gpurun_out/probe/partition_probe.txt
