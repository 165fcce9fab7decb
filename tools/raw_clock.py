"""Per-wave timeline of the fused buffer-index pass (k_raw_pass) at config 3
(abnn_debug_raw_wave_clock, 100-MHz ticks, relative to the earliest entry):
stream start / end, look-back, walk and end; the balance within and across
workgroups; and, over CLOCK_PASSES consecutive passes, how much of a
workgroup's lateness persists from one pass to the next (what the adaptive
partition can remove).  usage: python tools/raw_clock.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from abnn_amd import _lib  # noqa: E402

lib = _lib.load()
lib.abnn_debug_raw_fused(1)
P = int(os.environ.get("CLOCK_PASSES", "8"))
out = bench.raw_run("c3", 0, 20, 10, int(os.environ.get("STEPS", "30")), clock_passes=P)
W = out.pop("_wave_clocks").astype(np.int64)
print("timed: pass %.1f us  gate %.1f us" % (out["roofline"]["pass_ms_events"] * 1e3, out["roofline"]["avg_launch_ms"] * 1e3))
w = W[-1]
t0 = w[:, 0].min()
us = lambda x: (x - t0) / 100.0  # noqa: E731
names = ["entry", "stream start", "stream end", "look-back", "walk", "end"]
q = [0, 10, 50, 90, 99, 100]
print("last pass, us from entry" + "".join("%9s" % ("p%d" % p) for p in q))
for j, n in enumerate(names):
    print("%-24s" % n + "".join("%9.1f" % np.percentile(us(w[:, j]), p) for p in q))
dur = (w[:, 2] - w[:, 1]) / 100.0
print("%-24s" % "stream dur" + "".join("%9.1f" % np.percentile(dur, p) for p in q))
print("%-24s" % "iterations" + "".join("%9.0f" % np.percentile(w[:, 6], p) for p in q))
print("%-24s" % "survivors" + "".join("%9.0f" % np.percentile(w[:, 7], p) for p in q))
end = us(w[:, 2]).reshape(256, 16)
print("within-workgroup stream-end spread p50 %.1f p90 %.1f max %.1f" % tuple(np.percentile(end.max(1) - end.min(1), [50, 90, 100])))
print("workgroup last stream end p10 %.1f p50 %.1f p90 %.1f max %.1f" % tuple(np.percentile(end.max(1), [10, 50, 90, 100])))
# persistence: each pass's workgroup lateness (last stream end - the pass's median)
late = []
for p in range(P):
    e = ((W[p][:, 2] - W[p][:, 0].min()) / 100.0).reshape(256, 16).max(1)
    late.append(e - np.median(e))
late = np.array(late)
kernel = [((W[p][:, 5].max() - W[p][:, 0].min()) / 100.0) for p in range(P)]
print("kernel entry->end per pass (us):", " ".join("%.1f" % k for k in kernel))
if P > 1:
    r = [np.corrcoef(late[p], late[p + 1])[0, 1] for p in range(P - 1)]
    print("lateness std per pass:", " ".join("%.1f" % x for x in late.std(1)))
    print("pass-to-pass correlation of workgroup lateness:", " ".join("%.2f" % x for x in r))
    print("mean lateness over passes: std %.1f (persistent part)  max %.1f" % (late.mean(0).std(), late.mean(0).max()))
os.makedirs("gpurun_out", exist_ok=True)
np.save("gpurun_out/raw_clock.npy", W)
# the pass's end: per pass, the last tail (stream end), look-back, walk and
# wave end, and the workgroups that end last (stampers are the workgroups
# below the budget cut: their waves end after the look-back poll of every
# workgroup's word and the stamps)
print("per pass, us from entry: last stream end / look-back / walk / end;  latest-ending workgroups (wg: end, its last stream end, walk)")
for p in range(P):
    w = W[p].astype(np.int64)
    t0 = w[:, 0].min()
    u = (w - t0) / 100.0
    wg_end = u[:, 5].reshape(256, 16).max(1)
    wg_se = u[:, 2].reshape(256, 16).max(1)
    wg_walk = u[:, 4].reshape(256, 16).max(1)
    top = np.argsort(-wg_end)[:4]
    print("  %.1f / %.1f / %.1f / %.1f  " % (u[:, 2].max(), u[:, 3].max(), u[:, 4].max(), u[:, 5].max()) +
          "  ".join("wg%d: %.1f (%.1f, %.1f)" % (g, wg_end[g], wg_se[g], wg_walk[g]) for g in top))
stampers = W[-1][:, 5].reshape(256, 16).max(1) - W[-1][:, 4].reshape(256, 16).max(1) > 0
print("last pass: workgroups whose end follows their walk (stampers): %d; the latest stream end's workgroup: %d"
      % (int(stampers.sum()), int(np.argmax(((W[-1][:, 2] - W[-1][:, 0].min()) / 100.0).reshape(256, 16).max(1)))))
