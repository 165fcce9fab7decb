#!/bin/bash
# Round 4 GPU call Q: the committed tree -- whole -m gpu suite, rocprofv3
# trace + PMC traffic of config 3, wave timelines, the bench set, and an
# A/B of the partition's gain now that tails no longer go by wave age.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
t 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r4q_suite.log 2>&1 || { echo "suite failed"; tail -40 gpurun_out/r4q_suite.log; exit 1; }
tail -2 gpurun_out/r4q_suite.log
t 700 bash tools/profile.sh r04q c3 > gpurun_out/prof_r04q.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/prof_r04q.log; exit 1; }
tail -3 gpurun_out/prof_r04q.log
t 200 python3 tools/wc_multi.py 200 > gpurun_out/wcm_r04q.txt 2>&1 || echo "wcm failed"
b() { local name=$1; shift; t 300 python -u bench.py "$@" > gpurun_out/q_$name.json 2> gpurun_out/q_$name.err || { echo "bench $name failed"; tail -5 gpurun_out/q_$name.err; exit 1; }; python3 tools/bench_line.py gpurun_out/q_$name.json "$name"; }
b driver --steps 20 --warmup 5
b c3 --steps 200
b c3p --plasticity --steps 100 --no-cpu-baseline
b shard --shard-path --steps 200 --no-cpu-baseline
ROUNDS=3 t 300 bash tools/ab_cfg.sh g1=. g2=.,ABNN_ADAPT_GAIN=2 g3=.,ABNN_ADAPT_GAIN=3 > /dev/null || { echo "ab failed"; exit 1; }
cat gpurun_out/ab_cfg.txt
t 300 python3 tools/partition_probe.py 200 > gpurun_out/partition_probe.txt 2>&1 || echo "probe failed"; cat gpurun_out/partition_probe.txt
