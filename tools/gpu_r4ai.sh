#!/bin/bash
# Round 4 GPU call AI: the PMC traffic records restamped on the final
# sources (a header comment changed), with the default bench beside them.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
t 700 bash tools/profile.sh r04ai c3 > gpurun_out/prof_r04ai.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/prof_r04ai.log; exit 1; }
t 900 bash tools/profile_raw.sh r04ai_raw > gpurun_out/prof_r04ai_raw.log 2>&1 || { echo "raw profile failed"; tail -20 gpurun_out/prof_r04ai_raw.log; exit 1; }
t 400 python -u bench.py > gpurun_out/ai_default.json 2> gpurun_out/ai_default.err || { echo "bench failed"; tail -5 gpurun_out/ai_default.err; exit 1; }
python3 tools/bench_line.py gpurun_out/ai_default.json default
