#!/bin/bash
# Round 4 GPU call AK: the whole -m gpu suite and smoke() on the exact final tree.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
t 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/rak_suite.log 2>&1 || { echo "suite failed"; tail -40 gpurun_out/rak_suite.log; exit 1; }
tail -2 gpurun_out/rak_suite.log
t 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -1
