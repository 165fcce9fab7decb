#!/bin/bash
# rocprofv3 kernel trace + stats of one bench.py command line (no PMC):
# per-kernel durations for the breakdown of a mode's pass.
# usage: tools/prof_trace.sh TAG bench-args...   -> gpurun_out/prof_TAG/
set -o pipefail
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$out/trace" -o run -- \
    python3 bench.py "$@" > "$out/bench.json" 2> "$out/bench.err"
rc=$?
[ $rc -ne 0 ] && { echo "FATAL rc=$rc"; tail -5 "$out/bench.err"; exit 100; }
python3 - "$out" <<'PY'
import csv, glob, sys
out = sys.argv[1]
f = sorted(glob.glob(f"{out}/trace/**/*kernel_stats.csv", recursive=True))
if not f:
    print("no kernel_stats.csv"); sys.exit(0)
rows = list(csv.DictReader(open(f[0])))
for r in rows[:14]:
    print(f"{r['Name'][:70]:70s} calls {r['Calls']:>6s} avg_us {float(r['AverageNs'])/1e3:9.2f} total_ms {float(r['TotalDurationNs'])/1e6:9.2f} pct {float(r['Percentage']):6.2f}")
PY
