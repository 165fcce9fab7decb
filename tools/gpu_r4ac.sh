#!/bin/bash
# Round 4 GPU call AC: timing experiment only -- the reference-layout gate
# without its per-group refractory flush (wrong results: how much the
# per-group pipeline drain costs), interleaved with the committed library.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
for r in 1 2; do
  for lib in abnn_amd/libabnn_hip.so tools/exp/rawnoflush.so; do
    ABNN_LIB=$PWD/$lib t 300 python -u bench.py --raw --steps 50 > gpurun_out/br.json 2> gpurun_out/br.err || { echo "raw bench failed"; tail -5 gpurun_out/br.err; exit 1; }
    python3 tools/bench_line.py gpurun_out/br.json "raw $lib r$r"
  done
done | tee gpurun_out/raw_ab_ac.txt
