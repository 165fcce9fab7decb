#!/usr/bin/env python3
"""How fast the pass runs in the first seconds of a process on a box: blocks
of `every`-th-launch HIP-event timings over BLOCKS x 400 passes (config 3),
printed per block with the wall time since the graph was built.  Shows
whether a cold box (idle before the call) runs slower at first and for how
long -- what bench.py's default warm-up must cover.
usage: python tools/warm_curve.py [blocks]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from abnn_amd import CONFIGS, Brain  # noqa: E402

wl = CONFIGS["c3"]
blocks = int(sys.argv[1]) if len(sys.argv) > 1 else 40
b = Brain(wl.n_input, wl.n_output, wl.n_hidden, wl.n_syn, wl.events, device=0)
b.build_random_graph(1)
b.set_auto_stimulus(0, wl.n_input)
b.synchronize()
t0 = time.time()
for k in range(blocks):
    b.enable_timing(4)
    b.encode_traversal(400)
    b.synchronize()
    t = b.kernel_times() * 1e3
    print(f"block {k:3d} at {time.time() - t0:6.2f} s: median {np.median(t):6.1f} us  mean {t.mean():6.1f} us", flush=True)
