#!/bin/bash
# config 5 (4e9 records) on one GPU: sweep, then sweep with plasticity.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --config c5 --no-cpu-baseline > gpurun_out/b_c5.json 2> gpurun_out/b_c5.err || { tail -5 gpurun_out/b_c5.err; exit 1; }
timeout -k 10 600 python -u bench.py --config c5 --plasticity --no-cpu-baseline --steps 100 > gpurun_out/b_c5p.json 2>> gpurun_out/b_c5.err || { tail -5 gpurun_out/b_c5.err; exit 1; }
python3 - <<'PY'
import json
for f in ["gpurun_out/b_c5.json", "gpurun_out/b_c5p.json"]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    pl = d["config"].get("plasticity") or {}
    print(f, round(d["value"] / 1e9, 1), "G events/s", round(d["ms_per_step"], 4), "ms/pass", "frac", d["roofline"]["frac"],
          "n_syn", d["config"]["n_syn"], "pruned", pl.get("pruned"), "grown", pl.get("grown"))
PY
