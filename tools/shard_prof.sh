#!/bin/bash
# rocprofv3 kernel trace of the sharded pass at one GPU (bench.py --shard-path):
# per-kernel median duration and the gap after it, over the last passes.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_shard -o run -- \
    python3 bench.py --shard-path --no-cpu-baseline --steps 100 > gpurun_out/bench_shard_prof.json 2>&1 || { tail -5 gpurun_out/bench_shard_prof.json; exit 1; }
python3 - <<'PY'
import csv, glob, statistics
f = glob.glob("gpurun_out/prof_shard/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))[-300:]
per = {}
for a, b in zip(rows[:-1], rows[1:]):
    n = a["Kernel_Name"].split("(")[0].split("<")[0][-34:]
    per.setdefault(n, []).append(((int(a["End_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3,
                                  (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3))
for n, v in per.items():
    print(f"{n:36s} n={len(v):4d} dur median {statistics.median(x[0] for x in v):7.2f} us, gap after it {statistics.median(x[1] for x in v):7.2f} us")
PY
