#!/bin/bash
# SQ (shader sequencer) counters of the pass kernel on the GPU box: where the
# stream loop's issue slots go.  One rocprofv3 --pmc pass per group (at most
# 8 SQ counters each, MI355X_MICROARCH.md §rocprofv3 PMC slots), over
# tools/pass_times.py (config 3, 100 timed passes), medians per k_gate launch.
#   usage: tools/sq_profile.sh OUTFILE      (ABNN_LIB selects a variant library)
set -o pipefail
out=${1:-gpurun_out/sq.txt}
mkdir -p gpurun_out
export TMPDIR=/tmp
[ -f gpurun_out/counters_list.txt ] || timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
tools/pmc_pass.sh \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_LDS" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM" \
  "SQC_ICACHE_MISSES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT" | tee "$out"
