#!/bin/bash
# One GPU call for a kernel experiment on the in-tree library: a parity subset,
# then an interleaved knob A/B (tools/pass_times.py, 300 passes per run) and a
# per-wave timeline for each value.
#   KNOB=ABNN_X VALUES="0 1" [ROUNDS=2] [PARITY=1] [WC=1] bash tools/gpu_exp.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
(while sleep 50; do date +%s >> gpurun_out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
KNOB=${KNOB:-ABNN_NEXT_HELPERS}
if [ "${PARITY:-1}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plasticity.py -x -q --timeout 300 \
      --timeout-method thread > gpurun_out/exp_parity.txt 2>&1 || { tail -30 gpurun_out/exp_parity.txt; exit 1; }
  tail -1 gpurun_out/exp_parity.txt
fi
for r in $(seq 1 "${ROUNDS:-2}"); do
  for v in ${VALUES:-0 1}; do
    env "$KNOB=$v" timeout -k 10 120 python -u tools/pass_times.py 300 1 > gpurun_out/pt.txt 2>&1 || { tail -5 gpurun_out/pt.txt; exit 1; }
    printf "%s=%-5s r%s %s\n" "$KNOB" "$v" "$r" "$(grep launches gpurun_out/pt.txt | sed 's/.*us: //')"
  done
done | tee gpurun_out/exp_ab.txt
[ "${WC:-1}" = 1 ] || exit 0
for v in ${VALUES:-0 1}; do
  env "$KNOB=$v" B2B=1 timeout -k 10 120 python -u tools/wave_clock.py 120 > gpurun_out/exp_wc_$v.txt 2>&1 || { tail -5 gpurun_out/exp_wc_$v.txt; exit 1; }
  cp gpurun_out/wave_clock_p119.npy gpurun_out/exp_wc_$v.npy
  echo "== $KNOB=$v"; sed -n 2,20p gpurun_out/exp_wc_$v.txt
done
exit 0
