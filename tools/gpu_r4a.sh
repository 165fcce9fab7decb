set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_raw.py tests/test_cpp_api.py -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/raw_tests.log 2>&1 || { echo "raw tests failed"; tail -30 gpurun_out/raw_tests.log; exit 1; }
tail -3 gpurun_out/raw_tests.log
timeout -k 10 300 python -u bench.py --raw --steps 50 > gpurun_out/bench_raw.json 2> gpurun_out/bench_raw.err || { echo "raw bench failed"; tail -20 gpurun_out/bench_raw.err; exit 1; }
cat gpurun_out/bench_raw.json
timeout -k 10 240 python3 tools/pass_times.py 300 > gpurun_out/pt_base.txt 2>&1 && tools/sq_profile.sh gpurun_out/sq_base.txt && timeout -k 10 300 python3 tools/cpu_scaling.py 3 16 64 all > gpurun_out/cpu_scaling.txt 2>&1
