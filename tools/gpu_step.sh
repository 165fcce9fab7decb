#!/bin/bash
# Run one GPU step under its own time limit; stop the whole call on a crash,
# abort or timeout (exit codes other than 0 and 1), never retry.
# usage: tools/gpu_step.sh SECONDS LOGNAME cmd...
limit=$1; shift; log=$1; shift
mkdir -p gpurun_out
echo "== $(date +%T) $*" >> gpurun_out/steps.log
timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
rc=$?
echo "== rc=$rc $*" >> gpurun_out/steps.log
tail -5 "gpurun_out/$log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
  echo "FATAL step rc=$rc: stopping" ; exit 100
fi
exit 0
