#!/bin/bash
# GPU box: the -m gpu suite, the smoke test and a default bench run, each step
# under its own time limit, stopping at the first failure.  A heartbeat file
# under gpurun_out/ marks the long oracle-bound tests as alive.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
(while sleep 50; do date +%s >> gpurun_out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
sel=${TESTS:-tests}
timeout -k 10 ${SUITE_LIMIT:-1000} python -u -m pytest $sel -m gpu -x -v --timeout 700 --timeout-method thread \
    ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
[ "${SMOKE:-1}" = 1 ] && { timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }; tail -2 gpurun_out/smoke.log; }
[ "${BENCH:-1}" = 1 ] && { timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }; cat gpurun_out/bench.json; }
exit 0
