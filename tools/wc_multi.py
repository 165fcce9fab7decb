#!/usr/bin/env python3
"""Per-wave timelines of the last 8 back-to-back fused passes beside their
HIP-event launch times (every launch timed): where a pass's time goes, and
how much of the launch lies outside the waves (dispatch, the kernel's end).
Times are us from the pass's first wave entry.
usage: python tools/wc_multi.py [passes]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from abnn_amd import CONFIGS, Brain  # noqa: E402

wl = CONFIGS[os.environ.get("CFG", "c3")]
passes = int(sys.argv[1]) if len(sys.argv) > 1 else 200
events = int(os.environ.get("EVENTS", wl.events))  # EVENTS=1000000000: the full sweep
b = Brain(wl.n_input, wl.n_output, wl.n_hidden, wl.n_syn, events, device=0)
b.build_random_graph(1)
if hasattr(b._lib, "abnn_debug_set_wave_clock"):  # the timeline is recorded on request only
    b._lib.abnn_debug_set_wave_clock(b._h, 1)
b.set_auto_stimulus(0, wl.n_input)
b.encode_traversal(74)
b.synchronize()
b.enable_timing(1)
b.encode_traversal(passes)
b.synchronize()
t = b.kernel_times() * 1e3
p_last = b.scalars()["pass_index"] - 1
nr, KW = 16384, 16
f = b._lib.abnn_debug_wave_clock_slot
f.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
f.restype = ctypes.c_int
rows = []
print(f"launch times (HIP events) of all {len(t)}: median {np.median(t):.1f} mean {t.mean():.1f} us")
print("pass  launch  span | stream end p50/p90/max | tail end p50/max | lookback max | walk max | seen max | exit p50/max")
for k in range(7, -1, -1):
    p = p_last - k
    buf = np.zeros(KW * nr, dtype=np.uint64)
    assert f(b._h, p % 8, buf.ctypes.data, buf.size) == 0
    w = buf.reshape(-1, KW).astype(np.int64)
    w = w[w[:, 0] > 0]
    e0 = w[:, 3].min()
    us = lambda c: (w[:, c] - e0) * 1e-2  # noqa: E731
    se, en, lb, wk = us(1), us(2), us(4), us(5)
    w0 = w[::16]
    ex = (w0[:, 13] - e0) * 1e-2
    seen = (w0[w0[:, 12] > 0, 12] - e0) * 1e-2
    lt = t[len(t) - 1 - k]
    span = ex.max()
    rows.append((lt, span))
    print(f"{p:5d} {lt:6.1f} {span:6.1f} | {np.median(se):5.1f} {np.percentile(se, 90):5.1f} {se.max():5.1f} | "
          f"{np.median(en):5.1f} {en.max():5.1f} | {lb.max():5.1f} | {wk.max():5.1f} | "
          f"{seen.max() if len(seen) else 0:5.1f} | {np.median(ex):5.1f} {ex.max():5.1f}")
    np.save(os.path.join(os.environ.get("OUT", "gpurun_out"), f"wcm_p{k}.npy"), w)
    rw = us(14)
    if k == 0:
        ct, nc, st = w[:, 6] * 1e-2, w[:, 7], us(1) - us(0)
        print("   last pass: per wave stream (start->stream end) pcts 50/90/max", np.round(np.percentile(st, [50, 90, 100]), 1),
              " mid-stream chunks", np.round(np.percentile(nc, [50, 90, 100]), 1),
              " chunk time us", np.round(np.percentile(ct, [50, 90, 100]), 1),
              " tail us", np.round(np.percentile(en - se, [50, 90, 100]), 1),
              " survivors", np.round(np.percentile(w[:, 8], [50, 90, 100]), 0))
        m = w[:, 14] > 0
        print("   last pass: range_walk dur pcts 50/90/99/max", np.round(np.percentile((rw - lb)[m], [50, 90, 99, 100]), 1),
              " lds walk+items dur", np.round(np.percentile((wk - rw)[m], [50, 90, 99, 100]), 1))
        w0m = (np.arange(len(w)) % 16 == 0) & (w[:, 12] > 0)
        if w0m.any():
            sn = (w[:, 12] - e0) * 1e-2
            print("   stamping wave 0: seen - lb", np.round(np.percentile((sn - lb)[w0m], [50, 90, 100]), 1),
                  " range_walk", np.round(np.percentile((rw - sn)[w0m], [50, 90, 100]), 1),
                  " lds walk", np.round(np.percentile((wk - rw)[w0m], [50, 90, 100]), 1))
r = np.array(rows)
print(f"mean launch {r[:, 0].mean():.1f} us, mean wave span {r[:, 1].mean():.1f} us, outside the waves {r[:, 0].mean() - r[:, 1].mean():.1f} us")
