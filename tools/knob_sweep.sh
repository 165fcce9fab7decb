#!/bin/bash
# tools/pass_times.py (300 passes, every launch timed) for each value of one
# env knob, over the in-tree library and tools/exp/*.so.
# usage: tools/knob_sweep.sh KNOB v1 v2 ...
set -o pipefail
knob=$1; shift
libs=("abnn_amd/libabnn_hip.so" tools/exp/*.so)
for v in "$@"; do
  for lib in "${libs[@]}"; do
    [ -f "$lib" ] || continue
    env "$knob=$v" ABNN_LIB=$PWD/$lib timeout -k 10 120 python -u tools/pass_times.py 300 1 > gpurun_out/ks.txt 2>&1 || exit 1
    printf "%-14s %s=%-5s %s\n" "$(basename "$lib" .so)" "$knob" "$v" "$(grep launches gpurun_out/ks.txt | sed 's/.*us: //')"
  done
done
