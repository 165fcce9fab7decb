#!/bin/bash
# Counters of random-edge mode's gate (round 6, DESIGN.md §5 random mode):
# two --pmc passes of ≤ 2 TA / 4 TCC / 1 GRBM counters over a short random-mode
# bench, then per-launch sums of k_gate (tools/pmc_kernel.py).
# usage: tools/pmc_random.sh TAG
set -o pipefail
tag=${1:-r06}
out=gpurun_out/pmc_$tag
mkdir -p "$out"
export TMPDIR=/tmp
args="--mode random --steps 4 --warmup 2 --settle 6 --no-cpu-baseline --no-reference-layout"
timeout -s KILL 150 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE -T \
    --output-format csv -d "$out/ta" -o run -- python3 bench.py $args > "$out/ta.json" 2> "$out/ta.err" || { echo "FATAL ta"; exit 100; }
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum -T \
    --output-format csv -d "$out/tcc" -o run -- python3 bench.py $args > "$out/tcc.json" 2> "$out/tcc.err" || { echo "FATAL tcc"; exit 100; }
python3 tools/pmc_kernel.py "$out" k_gate | tee "$out/summary.txt"
