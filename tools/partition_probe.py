#!/usr/bin/env python3
"""The adaptive partition against what it balances: after N back-to-back
fused passes at config 3, every range's length (abnn_debug_range_bounds: the
bounds the NEXT pass uses and the ones the last pass used) beside the last
pass's per-range cost proxy (tail end - stream start, tools/wc_multi.py's
clocks), grouped by wave slot and by workgroup.
usage: python tools/partition_probe.py [passes]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from abnn_amd import CONFIGS, Brain  # noqa: E402

wl = CONFIGS[os.environ.get("CFG", "c3")]
passes = int(sys.argv[1]) if len(sys.argv) > 1 else 200
b = Brain(wl.n_input, wl.n_output, wl.n_hidden, wl.n_syn, wl.events, device=0)
b.build_random_graph(1)
if hasattr(b._lib, "abnn_debug_set_wave_clock"):  # the timeline is recorded on request only
    b._lib.abnn_debug_set_wave_clock(b._h, 1)
b.set_auto_stimulus(0, wl.n_input)
b.encode_traversal(passes)
b.synchronize()
nr, KW = 4096, 16
fb = b._lib.abnn_debug_range_bounds
fb.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
fb.restype = ctypes.c_int
fw = b._lib.abnn_debug_wave_clock_slot
fw.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
fw.restype = ctypes.c_int
rows = []
for k in range(6):  # one pass at a time: the bounds each pass used, then its clocks
    bounds = np.zeros(nr + 1, dtype=np.uint32)
    assert fb(b._h, bounds.ctypes.data, bounds.size) == 0
    b.encode_traversal(1)
    b.synchronize()
    p = b.scalars()["pass_index"] - 1
    buf = np.zeros(KW * 16384, dtype=np.uint64)
    assert fw(b._h, p % 8, buf.ctypes.data, buf.size) == 0
    w = buf.reshape(-1, KW)[:nr].astype(np.int64)
    e0 = w[:, 3].min()
    cost = (w[:, 2] - w[:, 0]) * 1e-2
    tend = (w[:, 2] - e0) * 1e-2
    ln = np.diff(bounds.astype(np.int64))
    rows.append((ln, cost, tend))
    np.save(os.path.join(os.environ.get("OUT", "gpurun_out"), f"probe_{k}.npy"),
            np.concatenate([bounds.astype(np.int64), w[:, 0], w[:, 2], w[:, 7]]))
ln = np.array([r[0] for r in rows]).astype(float)
cost = np.array([r[1] for r in rows])
tend = np.array([r[2] for r in rows])
sl = np.arange(nr) % 16
print(f"after {passes} passes; {len(rows)} single passes probed")
print("slot:          " + " ".join(f"{i:6d}" for i in range(16)))
print("len / mean:    " + " ".join(f"{(ln[:, sl == i].mean() / ln.mean()):6.3f}" for i in range(16)))
print("cost dev us:   " + " ".join(f"{(cost[:, sl == i].mean() - cost.mean()):6.2f}" for i in range(16)))
print("tail end dev:  " + " ".join(f"{(tend[:, sl == i].mean() - tend.mean()):6.2f}" for i in range(16)))
dl = np.diff(ln, axis=0)
print("len change per pass by slot (iterations):", " ".join(f"{dl[:, sl == i].mean():5.2f}" for i in range(16)))
wg_t = tend.reshape(len(rows), 256, 16).max(2)
wg_l = ln.reshape(len(rows), 256, 16).sum(2)
d = wg_t - wg_t.mean(1, keepdims=True)
print("WG max tail end: corr pass to pass", [round(np.corrcoef(d[i], d[i + 1])[0, 1], 2) for i in range(len(rows) - 1)])
print("WG length change vs WG lateness (corr):", round(np.corrcoef(d[:-1].ravel(), np.diff(wg_l, axis=0).ravel())[0, 1], 3))
late = np.argsort(d.mean(0))[-5:]
print("latest WGs:", late.tolist(), "dev", d.mean(0)[late].round(2).tolist(), "len/mean", (wg_l.mean(0)[late] / wg_l.mean()).round(3).tolist())
