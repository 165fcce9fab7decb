#!/bin/bash
# Interleaved A/B of the in-tree library and tools/exp/*.so on one box:
# ROUNDS rounds of tools/pass_times.py (300 back-to-back passes, every launch
# timed) per library.  usage: tools/ab_times.sh [ROUNDS]
set -o pipefail
export ABNN_LIB_ANY_ABI=1  # variants of an older ABI (timing entry points only)
ROUNDS=${1:-3}
libs=("abnn_amd/libabnn_hip.so" tools/exp/*.so)
for r in $(seq 1 "$ROUNDS"); do
  for lib in "${libs[@]}"; do
    [ -f "$lib" ] || continue
    ABNN_LIB=$PWD/$lib timeout -k 10 120 python -u tools/pass_times.py 300 1 > gpurun_out/pt.txt 2>&1 || exit 1
    printf "%-22s r%s %s\n" "$(basename "$lib" .so)" "$r" "$(grep launches gpurun_out/pt.txt | sed 's/.*us: //')"
  done
done
