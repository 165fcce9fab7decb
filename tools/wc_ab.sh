#!/bin/bash
# Per-wave timelines (tools/wave_clock.py, back-to-back passes) of the in-tree
# library and every tools/exp/*.so, each saved as gpurun_out/wc_<name>.{txt,npy}.
set -o pipefail
libs=("abnn_amd/libabnn_hip.so" tools/exp/*.so)
for lib in "${libs[@]}"; do
  [ -f "$lib" ] || continue
  n=$(basename "$lib" .so)
  ABNN_LIB=$PWD/$lib B2B=1 timeout -k 10 120 python tools/wave_clock.py ${PASSES:-120} > "gpurun_out/wc_$n.txt" 2>&1 || exit 1
  mv gpurun_out/wave_clock_p*.npy "gpurun_out/wc_$n.npy"
done
