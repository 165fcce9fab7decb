#!/bin/bash
# Round 4 GPU call M: the whole -m gpu suite on the in-tree library (tail
# priority 3, DMA-only prologue wait, next-image zeroing at the pass end),
# then the committed evidence: rocprofv3 trace + PMC traffic of config 3.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
t() { timeout -k 10 "$@"; }
t 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r4m_suite.log 2>&1 || { echo "suite failed"; tail -40 gpurun_out/r4m_suite.log; exit 1; }
tail -3 gpurun_out/r4m_suite.log
