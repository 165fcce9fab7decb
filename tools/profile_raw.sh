#!/bin/bash
# The rocprofv3 evidence for the reference-layout path (bench.py --raw):
#   1. --kernel-trace --stats      -> per-kernel durations
#   2. --pmc FETCH_SIZE, 3. --pmc WRITE_SIZE (separate passes)
#   4. tools/pmc_summary.py ... k_raw_pass -> profiles/traffic_raw_c3.json (KERNEL=k_raw_gate
#      with ABNN_RAW_FUSED=0)
# usage: tools/profile_raw.sh TAG
set -o pipefail
tag=${1:-r04x_raw}
out=gpurun_out/prof_$tag
mkdir -p "$out" profiles
export TMPDIR=/tmp
run() { timeout -k 10 420 "$@"; rc=$?; if [ $rc -ne 0 ]; then echo "FATAL rc=$rc: $*"; exit 100; fi; }
run rocprofv3 --kernel-trace --stats -T --output-format csv -d "$out/trace" -o run -- \
    python3 bench.py --raw --steps 100 --warmup 10 > "$out/bench_trace.json"
run rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$out/fetch" -o run -- \
    python3 bench.py --raw --steps 10 --warmup 10 > "$out/bench_fetch.json"
run rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$out/write" -o run -- \
    python3 bench.py --raw --steps 10 --warmup 10 > "$out/bench_write.json"
python3 tools/pmc_summary.py "$out" "$tag" raw_c3 "${KERNEL:-k_raw_pass}"
