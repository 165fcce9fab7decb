#!/bin/bash
# Round 4 GPU call Z: the in-place compaction in rounds of two blocks with
# LDS-only scan barriers, and the grown records appended by 1024-slot blocks
# in parallel -- plasticity parity, c3p/c5p against the committed library,
# and the new update's kernel times.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/z
t() { timeout -k 10 "$@"; }
t 900 python -u -m pytest tests/test_gpu_plasticity.py tests/test_gpu_parity.py tests/test_sharded_gpu.py tests/test_gpu_scale.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r4z_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4z_tests.log; exit 1; }
tail -2 gpurun_out/r4z_tests.log
for r in 1 2; do
  for lib in tools/exp/devupd.so abnn_amd/libabnn_hip.so; do
    ABNN_LIB=$PWD/$lib t 300 python -u bench.py --plasticity --steps 200 --no-cpu-baseline > gpurun_out/bp.json 2> gpurun_out/bp.err || { echo "c3p bench failed"; tail -5 gpurun_out/bp.err; exit 1; }
    python3 tools/bench_line.py gpurun_out/bp.json "c3p $lib r$r"
  done
done | tee gpurun_out/c3p_ab_z.txt
for lib in tools/exp/devupd.so abnn_amd/libabnn_hip.so; do
  ABNN_LIB=$PWD/$lib t 400 python -u bench.py --config c5 --plasticity --steps 100 --no-cpu-baseline > gpurun_out/bp5.json 2> gpurun_out/bp5.err || { echo "c5p bench failed"; tail -5 gpurun_out/bp5.err; exit 1; }
  python3 tools/bench_line.py gpurun_out/bp5.json "c5p $lib"
done | tee -a gpurun_out/c3p_ab_z.txt
t 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/z/c3p -o run -- python3 bench.py --plasticity --steps 200 --no-cpu-baseline > gpurun_out/z/c3p.json 2> gpurun_out/z/c3p.err || { echo "prof failed"; tail -5 gpurun_out/z/c3p.err; exit 1; }
cut -d, -f1-7 gpurun_out/z/c3p/run_kernel_stats.csv | head -16
