#!/bin/bash
# Round 4 GPU call C: the raw launcher's tests + bench after the two-level
# scan; interleaved A/B of batched filter reads (with / without stamps after
# the walk); SQ counters of the batched variant.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
t 400 python -u -m pytest tests/test_gpu_raw.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4c_raw.log 2>&1 || { echo "raw tests failed"; tail -30 gpurun_out/r4c_raw.log; exit 1; }
tail -2 gpurun_out/r4c_raw.log
t 200 python -u bench.py --raw --steps 50 > gpurun_out/bench_raw.json 2> gpurun_out/bench_raw.err || { echo "raw bench failed"; tail -20 gpurun_out/bench_raw.err; exit 1; }
python3 -c "import json; b=json.load(open('gpurun_out/bench_raw.json')); print('raw', b['ms_per_step'], b['roofline']['avg_launch_ms'], b['roofline']['frac'])"
ROUNDS=3 t 500 bash tools/ab_cfg.sh noknobs=tools/exp/noknobs.so sf=tools/exp/stampfirst.so lds=tools/exp/ldsbatch.so lds_sf=tools/exp/ldsbatch_sf.so > /dev/null || { echo "ab failed"; exit 1; }
cat gpurun_out/ab_cfg.txt
ABNN_LIB=$PWD/tools/exp/ldsbatch.so t 300 tools/sq_profile.sh gpurun_out/sq_ldsbatch.txt > /dev/null || { echo "sq failed"; exit 1; }
