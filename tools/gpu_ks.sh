#!/bin/bash
# knob sweep on the in-tree library (rebuilt from the tree by the parity run's
# conftest when stale): interleaved pass times for each value.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
(while sleep 50; do date +%s >> gpurun_out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
python -c "from abnn_amd.build import build_hip; build_hip()" || exit 1
KNOB=${KNOB:-ABNN_SPEC_MARGIN}
for r in 1 2; do
  for v in ${VALUES:--1 8 16 32 64}; do
    env "$KNOB=$v" timeout -k 10 120 python -u tools/pass_times.py 300 1 > gpurun_out/ks.txt 2>&1 || { tail -5 gpurun_out/ks.txt; exit 1; }
    printf "%s=%-5s r%s %s\n" "$KNOB" "$v" "$r" "$(grep launches gpurun_out/ks.txt | sed 's/.*us: //')"
  done
done | tee gpurun_out/ks_sweep.txt
