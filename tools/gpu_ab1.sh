#!/bin/bash
# A/B of kernel variants on one box: parity subset of the newest variant,
# interleaved pass times, a knob sweep and per-wave timelines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
(while sleep 50; do date +%s >> gpurun_out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
NEW=${NEW:-tools/exp/tl.so}
ABNN_LIB=$PWD/$NEW timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random.py -x -q --timeout 300 --timeout-method thread -k "config1 or c2_lite or edge_cases or pass_variants or virtual_shards or collisions" > gpurun_out/ab_parity.txt 2>&1 || { tail -30 gpurun_out/ab_parity.txt; exit 1; }
tail -2 gpurun_out/ab_parity.txt
bash tools/ab_times.sh 3 2>&1 | tee gpurun_out/ab1.txt || exit 1
for lib in abnn_amd/libabnn_hip.so $NEW; do
  ABNN_LIB=$PWD/$lib B2B=1 timeout -k 10 120 python -u tools/wave_clock.py 120 > gpurun_out/wc_$(basename $lib .so).txt 2>&1 || exit 1
  echo "== $lib"; sed -n 2,14p gpurun_out/wc_$(basename $lib .so).txt
done
[ "${RAW:-1}" = 1 ] && { timeout -k 10 300 python -u tools/raw_bench.py 50 > gpurun_out/raw_bench.txt 2>&1 || { tail -5 gpurun_out/raw_bench.txt; exit 1; }; tail -1 gpurun_out/raw_bench.txt; }
exit 0
