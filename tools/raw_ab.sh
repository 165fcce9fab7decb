#!/bin/bash
# Interleaved A/B of the reference-layout pass (bench.py --raw, config 3):
# the in-tree library and every tools/exp/*.so, ROUNDS rounds on one box.
# usage (GPU box): ROUNDS=2 bash tools/raw_ab.sh [extra bench args]
set -o pipefail
export TMPDIR=/tmp
export ABNN_LIB_ANY_ABI=1
mkdir -p gpurun_out
libs=("abnn_amd/libabnn_hip.so" tools/exp/*.so)
for r in $(seq 1 "${ROUNDS:-2}"); do
  for lib in "${libs[@]}"; do
    [ -f "$lib" ] || continue
    n=$(basename "$lib" .so)
    ABNN_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --raw --no-cpu-baseline "$@" > gpurun_out/rawab_${n}_$r.txt 2>&1 \
      || { tail -20 gpurun_out/rawab_${n}_$r.txt; exit 1; }
    python3 tools/bench_line.py gpurun_out/rawab_${n}_$r.txt "raw $n r$r"
  done
done | tee gpurun_out/raw_ab.txt
