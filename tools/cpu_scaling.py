#!/usr/bin/env python3
"""Thread scaling of the CPU baseline (bench.py cpu_baseline: the threaded C
oracle on config 3's first E synapses, the only ones a sweep pass touches):
one graph, settled once, then `passes` timed passes at each thread count.
usage: python tools/cpu_scaling.py [passes] [threads ...]   (default 3; 16 64 all)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from abnn_amd import CONFIGS  # noqa: E402
from bench import SETTLE_PASSES, host_cpus  # noqa: E402
from oracle import oracle as O  # noqa: E402

wl = CONFIGS["c3"]
passes = int(sys.argv[1]) if len(sys.argv) > 1 else 3
hc = host_cpus()
avail = hc["available"]
counts = [int(x) if x != "all" else avail for x in (sys.argv[2:] or ["16", "64", "all"])]
E = O.visited_events(wl.events, wl.n_syn)
ob = O.OracleBrain(wl.n_input, wl.n_output, wl.n_hidden, E, wl.events)
t = time.perf_counter()
ob.build_random_graph(1, nthreads=min(avail, 256))
ob.set_auto_stimulus(0, wl.n_input)
ob.pass_threaded(SETTLE_PASSES, nthreads=min(avail, 256))
print(f"host: {hc}; graph {E:,} synapses + {SETTLE_PASSES} settle passes in {time.perf_counter() - t:.1f} s",
      flush=True)
for n in counts:
    n = max(1, min(n, 256))
    t = time.perf_counter()
    ob.pass_threaded(passes, nthreads=n)
    dt = time.perf_counter() - t
    print(f"threads {n:4d}: {passes * E / dt / 1e9:7.3f} G events/s ({dt / passes * 1e3:.1f} ms per pass)", flush=True)
