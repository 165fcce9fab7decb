#!/usr/bin/env python3
"""Per-wave timeline of the gate kernel (diagnostics, always recorded).

Runs config 3 for `warm` passes, then reads the last pass's per-wave clocks
{start, stream done, end} (100 MHz s_memrealtime) and prints the spread of
start, stream-end and end times, the tail (refractory stage) durations and the
latest waves.  usage: [B2B=1] python tools/wave_clock.py [passes [first printed]]
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
if hasattr(b._lib, "abnn_debug_set_wave_clock"):  # the timeline is recorded on request only
    b._lib.abnn_debug_set_wave_clock(b._h, 1)
b.set_auto_stimulus(0, wl.n_input)
passes = int(sys.argv[1]) if len(sys.argv) > 1 else 12
first = int(sys.argv[2]) if len(sys.argv) > 2 else 0  # print passes >= first
b2b = os.environ.get("B2B", "0") == "1"  # passes back to back (as the bench runs them): only the last is printed
if b2b:
    b.encode_traversal(passes - 1)
for p in range(passes - 1 if b2b else 0, passes):
    b.encode_traversal(1)
    b.synchronize()
    if p < first:
        continue
    nr, KW = 16384, 16  # kWaveClock u64 per range (engine.h)
    buf = np.zeros(KW * nr + 32, dtype=np.uint64)
    f = b._lib.abnn_debug_wave_clock
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    f.restype = ctypes.c_int
    assert f(b._h, buf.ctypes.data, buf.size) == 0
    w = buf[:KW * nr].reshape(-1, KW).astype(np.int64)
    w = w[w[:, 0] > 0]
    t0 = w[:, 0].min()
    print(f"  entry (before the filter load) to start: " + " ".join(
        f"{v:5.2f}" for v in np.percentile((w[:, 0] - w[:, 3]) * 10e-3, [0, 50, 100])) +
        f" us; first entry {(w[:, 3].min() - t0) * 10e-3:.2f} us; last end - first entry {(w[:, 2].max() - w[:, 3].min()) * 10e-3:.2f} us")
    st, se, en = (w[:, 0] - t0) * 10e-3, (w[:, 1] - t0) * 10e-3, (w[:, 2] - t0) * 10e-3  # us
    q = lambda x: " ".join(f"{v:7.1f}" for v in np.percentile(x, [0, 10, 50, 90, 99, 100]))
    print(f"pass {p}: waves {len(w)}   percentiles 0/10/50/90/99/100 (us)")
    print(f"  start       {q(st)}")
    print(f"  stream end  {q(se)}")
    print(f"  end         {q(en)}")
    print(f"  stream dur  {q(se - st)}")
    print(f"  tail dur    {q(en - se)}")
    ct = w[:, 6] * 10e-3
    print(f"  mid-stream refractory chunks: {int(w[:, 7].sum())} in total, per wave max {int(w[:, 7].max())}; "
          f"time per wave {q(ct)}")
    print(f"  stream dur less chunks {q(se - st - ct)}")
    if (w[:, 5] > 0).all():  # fused pass: look-back done, walk done
        lb, wk = (w[:, 4] - t0) * 10e-3, (w[:, 5] - t0) * 10e-3
        print(f"  lookback at {q(lb)}")
        print(f"  walk done   {q(wk)}")
        print(f"  lb wait     {q(lb - en)}")
        print(f"  walk dur    {q(wk - lb)}")
        w0 = w[::16]  # wave 0 of each workgroup: all words seen (stampers), exit
        if (w0[:, 13] > 0).all():
            seen, ex = (w0[:, 12] - t0) * 10e-3, (w0[:, 13] - t0) * 10e-3
            stampers = w0[:, 12] > 0
            print(f"  wg exit     {q(ex)}")
            if stampers.any():
                print(f"  all words seen (stamping wgs: {int(stampers.sum())}) {q(seen[stampers])}")
    np.save(os.path.join(os.environ.get("OUT", "gpurun_out"), f"wave_clock_p{p}.npy"), w)
    rb = np.zeros(len(w) + 1, dtype=np.uint32)
    g = b._lib.abnn_debug_range_bounds
    g.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    g.restype = ctypes.c_int
    assert g(b._h, rb.ctypes.data, rb.size) == 0
    ln = np.diff(rb.astype(np.int64))  # bounds for the NEXT pass
    wid = np.arange(len(w)) % 16
    print("  next lengths r0..11:", ln[:12].tolist(), " per age group mean len:",
          [round(float(ln[(wid // 4) == a].mean()), 1) for a in range(4)],
          " per age group mean end:", [round(float(en[(wid // 4) == a].mean()), 1) for a in range(4)])
    late = np.argsort(en)[-6:]
    print("  latest waves (range: start/stream-end/end us):",
          "  ".join(f"{i}:{st[i]:.1f}/{se[i]:.1f}/{en[i]:.1f}" for i in late))
