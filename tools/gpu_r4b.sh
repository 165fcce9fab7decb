#!/bin/bash
# Round 4 GPU call B: interleaved A/B of the fused pass (round-3 kernel, dead
# knobs compiled out, stamps after the walk), SQ counters of the first and
# the last, the wave timelines, the CPU baseline's thread scaling.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
ROUNDS=3 t 500 bash tools/ab_cfg.sh base=tools/exp/base.so noknobs=tools/exp/noknobs.so stampfirst=tools/exp/stampfirst.so > /dev/null || { echo "ab failed"; exit 1; }
cat gpurun_out/ab_cfg.txt
ABNN_LIB=$PWD/tools/exp/base.so t 300 tools/sq_profile.sh gpurun_out/sq_base.txt > /dev/null || { echo "sq base failed"; exit 1; }
ABNN_LIB=$PWD/tools/exp/stampfirst.so t 300 tools/sq_profile.sh gpurun_out/sq_stampfirst.txt > /dev/null || { echo "sq new failed"; exit 1; }
ABNN_LIB=$PWD/tools/exp/stampfirst.so t 200 python3 tools/wc_multi.py 200 > gpurun_out/wcm_stampfirst.txt 2>&1 || echo "wcm failed"
t 300 python3 tools/cpu_scaling.py 3 16 64 all > gpurun_out/cpu_scaling.txt 2>&1 || echo "cpu scaling failed"
t 120 tools/ubench_random > gpurun_out/ubench_random.txt 2>&1 || echo "ubench random failed"
