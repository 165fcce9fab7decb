#!/bin/bash
# Round 4 GPU call AJ: SQ counters of the final pass kernel (tools/sq_profile.sh).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 bash tools/sq_profile.sh gpurun_out/sq_final.txt > gpurun_out/sq_final.log 2>&1 || { echo "sq failed"; tail -20 gpurun_out/sq_final.log; exit 1; }
cat gpurun_out/sq_final.txt
