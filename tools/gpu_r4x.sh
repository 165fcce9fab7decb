#!/bin/bash
# Round 4 GPU call X: PMC traffic for the reference-layout path
# (tools/profile_raw.sh -> k_raw_gate), and an A/B of the fused pass's end
# with fewer dirty lines (lightend: zeroing stores non-temporal, no wave
# clocks) against the committed library.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
t 900 bash tools/profile_raw.sh r04x_raw > gpurun_out/prof_r04x_raw.log 2>&1 || { echo "raw profile failed"; tail -20 gpurun_out/prof_r04x_raw.log; exit 1; }
tail -3 gpurun_out/prof_r04x_raw.log
ROUNDS=4 t 500 bash tools/ab_cfg.sh base=. lightend=tools/exp/lightend.so > /dev/null || { echo "ab failed"; exit 1; }
cat gpurun_out/ab_cfg.txt
