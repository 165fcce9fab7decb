#!/bin/bash
# Round 4 GPU call P: where the sharded pass's extra 1.3 us with the new
# shard walk comes from -- rocprofv3 kernel stats of the sharded pass for the
# committed library, items-only and items + shard walk, and their per-
# workgroup walk timelines (tools/shard_clock.py).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/p
t() { timeout -k 10 "$@"; }
for v in t3pro_c items itemsw; do
  ABNN_LIB=$PWD/tools/exp/$v.so t 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/p/$v -o run -- python3 bench.py --shard-path --steps 200 --no-cpu-baseline > gpurun_out/p/$v.json 2> gpurun_out/p/$v.err || { echo "prof $v failed"; tail -5 gpurun_out/p/$v.err; exit 1; }
  echo "== $v"; grep -E "k_gate|k_shard_walk|ncclDevKernel|AllGather" gpurun_out/p/$v/run_kernel_stats.csv | cut -d, -f1-4
  ABNN_LIB=$PWD/tools/exp/$v.so t 200 python3 tools/shard_clock.py 100 2>&1 | grep -v amdgpu.ids | tail -8
done
