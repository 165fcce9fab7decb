#!/bin/bash
# VGPRs / scratch / LDS of every kernel of the HIP library (the stream loop
# must not spill: a spilled in-flight load register drains every load).
cd "$(dirname "$0")/.." || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -c abnn_amd/csrc/kernels.hip \
    -o /tmp/abnn_k.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  python3 -c '
import re, sys
cur = None
for ln in sys.stdin:
    m = re.search(r"Function Name: (\S+)", ln)
    if m:
        cur = m.group(1)
        n = re.sub(r"_ZN4abnn12_GLOBAL__N_1\d+", "", cur)
        print(n[:60].ljust(60), end="")
        continue
    for k in ("VGPRs:", "ScratchSize [bytes/lane]:", "LDS Size [bytes/block]:"):
        if k in ln:
            print(" ", k.split()[0], ln.split(k)[1].split()[0], end="")
            if k.startswith("LDS"): print()
'
