#!/bin/bash
# Interleaved A/B of library/knob configurations on one box: ROUNDS rounds of
# tools/pass_times.py (300 back-to-back passes, every launch timed) per
# configuration.  A configuration is NAME=LIB[,VAR=VALUE...] (LIB relative
# to the repo; "." = the in-tree library).
#   ROUNDS=2 bash tools/ab_cfg.sh head=tools/exp/r03c.so new=. new_d0=.,ABNN_DEFER_STAMPS=0
set -o pipefail
export TMPDIR=/tmp
export ABNN_LIB_ANY_ABI=1  # variants of an older ABI (timing entry points only)
mkdir -p gpurun_out
for r in $(seq 1 "${ROUNDS:-2}"); do
  for cfg in "$@"; do
    name=${cfg%%=*}; rest=${cfg#*=}
    lib=${rest%%,*}; envs=""
    [ "$rest" != "$lib" ] && envs=$(echo "${rest#*,}" | tr ',' ' ')
    [ "$lib" = "." ] && lib=abnn_amd/libabnn_hip.so
    env ABNN_LIB=$PWD/$lib $envs timeout -k 10 120 python -u tools/pass_times.py 300 1 > gpurun_out/pt.txt 2>&1 || { tail -5 gpurun_out/pt.txt; exit 1; }
    printf "%-14s r%s %s\n" "$name" "$r" "$(grep launches gpurun_out/pt.txt | sed 's/.*us: //')"
  done
done | tee gpurun_out/ab_cfg.txt
