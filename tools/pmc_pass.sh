#!/bin/bash
# One rocprofv3 --pmc pass per argument group over tools/pass_times.py (100
# back-to-back passes), each under its own time limit; per-counter medians
# over the k_gate launches.   usage: tools/pmc_pass.sh "C1 C2" "C3 C4" ...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for grp in "$@"; do
  i=$((i+1)); out=gpurun_out/pmc_$i
  timeout -s KILL 120 rocprofv3 --pmc $grp -T --output-format csv -d $out -o run -- python3 tools/pass_times.py 100 > $out.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $out.log; exit 1; }
  python3 - "$out" <<'PY'
import csv, glob, statistics, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
v = {}
for r in csv.DictReader(open(f)):
    if "k_gate" in r["Kernel_Name"]:
        v.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, x in sorted(v.items()):
    print(f"{k:32s} median per launch {statistics.median(x[-60:]):14.0f}  (launches {len(x)})")
PY
done
