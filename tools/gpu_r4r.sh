#!/bin/bash
# Round 4 GPU call R: the partition probe with its raw arrays (bounds each
# pass used, stream start, tail end, full chunks per range) for an offline
# replay of the controller.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/probe
t() { timeout -k 10 "$@"; }
OUT=gpurun_out/probe t 300 python3 tools/partition_probe.py 200 > gpurun_out/probe/partition_probe.txt 2>&1 || { echo "probe failed"; tail -5 gpurun_out/probe/partition_probe.txt; exit 1; }
cat gpurun_out/probe/partition_probe.txt
