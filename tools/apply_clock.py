#!/usr/bin/env python3
"""Per-workgroup timeline of k_apply (diagnostics, abnn_debug_apply_clock).

Runs config 3 for `passes` passes and prints, for the last ones, the spread
over workgroups of each checkpoint (us after the earliest workgroup entry):
entry, scalars + filter zeroing, walk prefix + partition, walk done, ticket, and
the finalizing workgroup's pass end.  usage: python tools/apply_clock.py [passes [first printed]]
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from abnn_amd import CONFIGS, Brain  # noqa: E402

wl = CONFIGS[os.environ.get("CFG", "c3")]
b = Brain(wl.n_input, wl.n_output, wl.n_hidden, wl.n_syn, wl.events, device=0)
b.build_random_graph(1)
b.set_auto_stimulus(0, wl.n_input)
passes = int(sys.argv[1]) if len(sys.argv) > 1 else 12
first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
f = b._lib.abnn_debug_apply_clock
f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
f.restype = ctypes.c_int
names = {0: "entry", 1: "scalars", 4: "loads", 7: "prefix", 2: "partition", 3: "walked", 5: "ticket"}
for p in range(passes):
    b.encode_traversal(1)
    b.synchronize()
    if p < first:
        continue
    buf = np.zeros(8 * 256, dtype=np.uint64)
    assert f(b._h, buf.ctypes.data, buf.size) == 0
    w = buf.reshape(-1, 8).astype(np.int64)
    t0 = w[:, 0].min()
    print(f"pass {p}: percentiles 0/10/50/90/100 (us after the first entry)")
    for j, n in names.items():
        x = (w[:, j] - t0) * 0.01
        print(f"  {n:10s} " + " ".join(f"{v:7.2f}" for v in np.percentile(x, [0, 10, 50, 90, 100])))
    last = int(np.argmax(w[:, 6]))
    print(f"  end (wg {last}) {(w[last, 6] - t0) * 0.01:7.2f}   slowest walk: wg {int(np.argmax(w[:, 3] - w[:, 2]))}"
          f" {(np.max(w[:, 3] - w[:, 2])) * 0.01:.2f} us")
