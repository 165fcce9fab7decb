#!/bin/bash
# One GPU call of this round, from named steps (each under its own time limit,
# the call stops at the first failure; tools/gpu_step.sh):
#   tests=<pytest selection>  parity tests (-m gpu)
#   ab=<rounds>               interleaved pass times: in-tree library vs tools/exp/*.so
#   sq=<name>                 SQ counters of the in-tree library -> gpurun_out/<name>
#   bench=<name>[:args]       bench.py -> gpurun_out/<name>.json
#   wc=<file>                 per-wave timelines of 8 fused passes (tools/wc_multi.py)
#   wcbase=<file> / benchbase=<name>[:args]   the same with tools/exp/base.so
#   cal=<file>                FETCH_SIZE calibration (tools/ubench_fetch_cal.hip, prebuilt)
#   absweep=<rounds>          full-sweep bench (1e9 events) per library, interleaved
#   rawab=<rounds>            buffer-index bench, fused pass vs five launches, interleaved
#   rawvar=<rounds>           fused buffer-index bench per library (in-tree, tools/exp/*.so), interleaved
#   prof=<tag> / profraw=<tag>  rocprofv3 kernel trace + FETCH/WRITE passes (tools/profile.sh, profile_raw.sh)
#   shardvar=<rounds>         sharded-path bench at world 1 per library (in-tree, tools/exp/*.so), interleaved
#   rawclk=<file>             per-range timeline of the fused buffer-index pass (tools/raw_clock.py)
#   benchv=<variant>:<name>[:args]  bench.py with tools/exp/<variant>.so -> gpurun_out/<name>.json
#   pt=<file>:<lib>[,VAR=VALUE...]    tools/pass_times.py (300 passes) with a library ("." in-tree) and knobs
#   trace=<tag>[:bench args]        rocprofv3 kernel trace + stats of bench.py (tools/prof_trace.sh)
#   pmcrandom=<tag>                 TA / TCC counters of random mode's gate (tools/pmc_random.sh)
#   smoke
# usage: tools/gpu_call.sh step [step ...]
set -o pipefail
export TMPDIR=/tmp
export ABNN_LIB_ANY_ABI=1  # A/B variants of an older ABI (timing entry points only)
mkdir -p gpurun_out
(while sleep 50; do date +%s >> gpurun_out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for st in "$@"; do
  key=${st%%=*}; val=${st#*=}
  case $key in
    tests) bash tools/gpu_step.sh 900 tests.log python -u -m pytest $val -m gpu -x -v --timeout 600 --timeout-method thread || exit 1
           grep -q " passed" gpurun_out/tests.log && ! grep -q " failed" gpurun_out/tests.log || { echo "TESTS FAILED"; exit 1; } ;;
    ab) bash tools/gpu_step.sh 900 ab.txt bash tools/ab_times.sh "$val" || exit 1; cat gpurun_out/ab.txt ;;
    sq) bash tools/gpu_step.sh 400 "$val.log" bash tools/sq_profile.sh "gpurun_out/$val" || exit 1 ;;
    bench) name=${val%%:*}; args=""; [ "$name" != "$val" ] && args=${val#*:}
           timeout -k 10 400 python -u bench.py $args > "gpurun_out/$name.json" 2> "gpurun_out/$name.err" || { echo "bench $name failed"; tail -5 "gpurun_out/$name.err"; exit 1; }
           python3 tools/bench_line.py "gpurun_out/$name.json" "$name" ;;
    wc) bash tools/gpu_step.sh 300 "$val" python -u tools/wc_multi.py || exit 1; cat "gpurun_out/$val" ;;
    wcsweep) EVENTS=1000000000 bash tools/gpu_step.sh 300 "$val" python -u tools/wc_multi.py 40 || exit 1; cat "gpurun_out/$val" ;;
    wcbase) ABNN_LIB=$PWD/tools/exp/base.so bash tools/gpu_step.sh 300 "$val" python -u tools/wc_multi.py || exit 1; cat "gpurun_out/$val" ;;
    benchbase) name=${val%%:*}; args=""; [ "$name" != "$val" ] && args=${val#*:}
           ABNN_LIB=$PWD/tools/exp/base.so timeout -k 10 400 python -u bench.py $args > "gpurun_out/$name.json" 2> "gpurun_out/$name.err" || { echo "bench $name failed"; tail -5 "gpurun_out/$name.err"; exit 1; }
           python3 tools/bench_line.py "gpurun_out/$name.json" "$name(base)" ;;
    benchv) var=${val%%:*}; rest=${val#*:}; name=${rest%%:*}; args=""; [ "$name" != "$rest" ] && args=${rest#*:}
           ABNN_LIB=$PWD/tools/exp/$var.so timeout -k 10 400 python -u bench.py $args > "gpurun_out/$name.json" 2> "gpurun_out/$name.err" || { echo "bench $name failed"; tail -5 "gpurun_out/$name.err"; exit 1; }
           python3 tools/bench_line.py "gpurun_out/$name.json" "$name($var)" ;;
    pt) name=${val%%:*}; cfg=${val#*:}; lib=${cfg%%,*}; envs=""; [ "$cfg" != "$lib" ] && envs=$(echo "${cfg#*,}" | tr ',' ' ')
        [ "$lib" = "." ] && lib=abnn_amd/libabnn_hip.so
        env ABNN_LIB=$PWD/$lib $envs timeout -k 10 120 python -u tools/pass_times.py 300 1 > "gpurun_out/$name" 2>&1 || { tail -5 "gpurun_out/$name"; exit 1; }
        cat "gpurun_out/$name" ;;
    trace) tag=${val%%:*}; args=""; [ "$tag" != "$val" ] && args=${val#*:}
           bash tools/gpu_step.sh 600 "trace_$tag.log" bash tools/prof_trace.sh "$tag" $args || exit 1; cat "gpurun_out/trace_$tag.log" ;;
    pmcrandom) bash tools/gpu_step.sh 400 "pmcrandom_$val.log" bash tools/pmc_random.sh "$val" || exit 1; cat "gpurun_out/pmcrandom_$val.log" ;;
    cal) bash tools/gpu_step.sh 300 fetch_cal.log timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T --kernel-trace --output-format csv -d gpurun_out/fcal -o run -- ./tools/ubench_fetch_cal || exit 1
         python3 tools/fetch_cal.py gpurun_out/fcal | tee "gpurun_out/$val" ;;
    absweep) for r in $(seq 1 "$val"); do for lib in abnn_amd/libabnn_hip.so tools/exp/*.so; do
               ABNN_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --events 1000000000 --steps 30 --no-cpu-baseline > gpurun_out/abs.json 2> gpurun_out/abs.err || { echo "sweep $lib failed"; tail -5 gpurun_out/abs.err; exit 1; }
               python3 tools/bench_line.py gpurun_out/abs.json "$(basename $lib .so) r$r"
             done; done | tee gpurun_out/absweep.txt ;;
    rawab) for r in $(seq 1 "$val"); do for f in 1 0; do
             ABNN_RAW_FUSED=$f timeout -k 10 300 python -u bench.py --raw --steps 50 > gpurun_out/rab.json 2> gpurun_out/rab.err || { echo "raw bench failed"; tail -5 gpurun_out/rab.err; exit 1; }
             python3 tools/bench_line.py gpurun_out/rab.json "raw fused=$f r$r"
           done; done | tee gpurun_out/rawab.txt ;;
    rawvar) for r in $(seq 1 "$val"); do for lib in abnn_amd/libabnn_hip.so tools/exp/*.so; do
             ABNN_LIB=$PWD/$lib ABNN_RAW_FUSED=1 timeout -k 10 300 python -u bench.py --raw --steps 50 > gpurun_out/rv.json 2> gpurun_out/rv.err || { echo "raw bench failed"; tail -5 gpurun_out/rv.err; exit 1; }
             python3 tools/bench_line.py gpurun_out/rv.json "raw $(basename $lib .so) r$r"
           done; done | tee gpurun_out/rawvar.txt ;;
    prof) bash tools/gpu_step.sh 1300 "prof_$val.log" bash tools/profile.sh "$val" c3 || exit 1 ;;
    profraw) bash tools/gpu_step.sh 1300 "profraw_$val.log" bash tools/profile_raw.sh "$val" || exit 1 ;;
    shardvar) for r in $(seq 1 "$val"); do for lib in abnn_amd/libabnn_hip.so tools/exp/*.so; do
             ABNN_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --shard-path --steps 200 --no-cpu-baseline > gpurun_out/sv.json 2> gpurun_out/sv.err || { echo "shard bench failed"; tail -5 gpurun_out/sv.err; exit 1; }
             python3 tools/bench_line.py gpurun_out/sv.json "shard $(basename $lib .so) r$r"
           done; done | tee gpurun_out/shardvar.txt ;;
    rawclk) bash tools/gpu_step.sh 300 "$val" python -u tools/raw_clock.py || exit 1; cat "gpurun_out/$val" ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
           tail -1 gpurun_out/smoke.log ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
