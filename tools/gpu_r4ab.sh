#!/bin/bash
# Round 4 GPU call AB: PMC traffic of the reference-layout path on the final
# sources (tools/profile_raw.sh), then a knob sweep of the fused pass on
# them (flush threshold, chunk penalty, speculation), interleaved.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
t 900 bash tools/profile_raw.sh r04ab_raw > gpurun_out/prof_r04ab_raw.log 2>&1 || { echo "raw profile failed"; tail -20 gpurun_out/prof_r04ab_raw.log; exit 1; }
ROUNDS=3 t 800 bash tools/ab_cfg.sh base=. flush256=.,ABNN_FLUSH_AT=256 pen300=.,ABNN_CHUNK_PENALTY=300 pen1200=.,ABNN_CHUNK_PENALTY=1200 spec2=.,ABNN_SPEC=2 > /dev/null || { echo "ab failed"; exit 1; }
cat gpurun_out/ab_cfg.txt
