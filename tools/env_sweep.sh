#!/bin/bash
# Per-pass launch times (tools/pass_times.py) under each env setting given as
# an argument ("A=1 B=2" per setting; "-" = defaults).
set -o pipefail
for v in "$@"; do
  [ "$v" = "-" ] && v="X_UNUSED=0"
  env $v timeout -k 10 120 python -u tools/pass_times.py 300 1 > gpurun_out/pt.txt 2>&1 || exit 1
  echo "$v $(grep launches gpurun_out/pt.txt | sed 's/.*us: //')"
done
