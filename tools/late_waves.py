#!/usr/bin/env python3
"""One line per pass: the gate's last wave end vs the 99th percentile, and the
latest ranges (diagnostics for the sweep partition).  usage: python tools/late_waves.py [passes]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from abnn_amd import CONFIGS, Brain  # noqa: E402

wl = CONFIGS[os.environ.get("CFG", "c3")]
b = Brain(wl.n_input, wl.n_output, wl.n_hidden, wl.n_syn, wl.events, device=0)
b.build_random_graph(1)
if hasattr(b._lib, "abnn_debug_set_wave_clock"):  # the timeline is recorded on request only
    b._lib.abnn_debug_set_wave_clock(b._h, 1)
b.set_auto_stimulus(0, wl.n_input)
f = b._lib.abnn_debug_wave_clock
f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
f.restype = ctypes.c_int
passes = int(sys.argv[1]) if len(sys.argv) > 1 else 60
b.encode_traversal(20)
ends, p99s = [], []
for p in range(20, passes):
    b.encode_traversal(1)
    buf = np.zeros(4 * 16384 + 16, dtype=np.uint64)
    assert f(b._h, buf.ctypes.data, buf.size) == 0
    w = buf[:4 * 16384].reshape(-1, 4)
    w = w[w[:, 0] > 0].astype(np.int64)
    t0 = w[:, 3].min()
    en = (w[:, 2] - t0) * 0.01
    st = (w[:, 1] - w[:, 0]) * 0.01
    late = np.argsort(en)[-4:][::-1]
    ends.append(en.max())
    p99s.append(np.percentile(en, 99))
    print(f"pass {p}: end max {en.max():6.1f} p99 {np.percentile(en, 99):6.1f} p50 {np.percentile(en, 50):6.1f}  late: " +
          " ".join(f"r{i}({en[i]:.0f},tail {en[i] - (w[i, 1] - t0) * 0.01:.0f})" for i in late))
print(f"mean max {np.mean(ends):.1f}  mean p99 {np.mean(p99s):.1f}")
