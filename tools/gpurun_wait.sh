#!/bin/bash
# gpurun, retried only while no GPU box or slot is free (exit 3: nothing ran,
# nothing was charged); any other outcome -- success, a failing command, a
# refusal -- is returned at once.  usage: tools/gpurun_wait.sh [gpurun args]
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 90
done
exit 3
