#!/bin/bash
# Round 4 GPU call F: the sharded pass at world 1 (gate + RCCL all-gather +
# walk), round-3 kernel vs this tree, interleaved.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
for r in 1 2 3; do
  for lib in tools/exp/base.so abnn_amd/libabnn_hip.so; do
    ABNN_LIB=$PWD/$lib t 200 python -u bench.py --shard-path --steps 200 --no-cpu-baseline > gpurun_out/bs.json 2> gpurun_out/bs.err || { echo "shard bench failed"; tail -5 gpurun_out/bs.err; exit 1; }
    python3 tools/bench_line.py gpurun_out/bs.json "$lib r$r"
  done
done | tee gpurun_out/shard_ab.txt
