#!/bin/bash
# Collect the rocprofv3 evidence for one bench configuration on the GPU box.
#   1. --kernel-trace --stats      -> per-kernel durations (profiles/<tag>_kernel_stats.csv)
#   2. --pmc FETCH_SIZE            -> separate pass
#   3. --pmc WRITE_SIZE            -> separate pass
#   4. tools/pmc_summary.py        -> profiles/traffic_<config>.json
# usage: [PMC=0] tools/profile.sh TAG [CONFIG]   (PMC=0: kernel trace only)
set -o pipefail
tag=${1:-r01}; cfg=${2:-c3}
out=gpurun_out/prof_$tag
mkdir -p "$out" profiles
export TMPDIR=/tmp
run() { timeout -k 10 420 "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FATAL rc=$rc: $*"; exit 100; fi; }
run rocprofv3 --kernel-trace --stats -T --output-format csv -d "$out/trace" -o run -- \
    python3 bench.py --config "$cfg" --steps 200 --warmup 10 --no-cpu-baseline > "$out/bench_trace.json"
if [ "${PMC:-1}" = 1 ]; then
run rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$out/fetch" -o run -- \
    python3 bench.py --config "$cfg" --steps 10 --warmup 10 --no-cpu-baseline > "$out/bench_fetch.json"
run rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$out/write" -o run -- \
    python3 bench.py --config "$cfg" --steps 10 --warmup 10 --no-cpu-baseline > "$out/bench_write.json"
fi
python3 tools/pmc_summary.py "$out" "$tag" "$cfg"
