#!/usr/bin/env python3
"""Launch-by-launch durations of the pass kernel (HIP events around every
`every`-th launch) after the settle passes: the distribution, its periodicity
(by pass mod 2/3/8) and the slowest launches.  usage: python tools/pass_times.py [passes [every]]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from abnn_amd import CONFIGS, Brain  # noqa: E402

wl = CONFIGS[os.environ.get("CFG", "c3")]
passes = int(sys.argv[1]) if len(sys.argv) > 1 else 400
every = int(sys.argv[2]) if len(sys.argv) > 2 else 1
b = Brain(wl.n_input, wl.n_output, wl.n_hidden, wl.n_syn, wl.events, device=0)
b.build_random_graph(1)
b.set_auto_stimulus(0, wl.n_input)
b.encode_traversal(74)
b.synchronize()
b.enable_timing(every)
b.encode_traversal(passes)
b.synchronize()
t = b.kernel_times() * 1e3  # us
q = lambda x: " ".join(f"{v:6.1f}" for v in np.percentile(x, [0, 10, 25, 50, 75, 90, 99, 100]))
print(f"{len(t)} launches (every {every}), percentiles 0/10/25/50/75/90/99/100 us: {q(t)}  mean {t.mean():.1f}")
for m in (2, 3, 8):
    print(f"  mean by launch mod {m}:", [round(float(t[i::m].mean()), 1) for i in range(m)])
print("  lag-1 correlation:", round(float(np.corrcoef(t[:-1], t[1:])[0, 1]), 3))
print("  first 64:", " ".join(f"{v:.0f}" for v in t[:64]))
slow = np.argsort(t)[-10:]
print("  slowest (index:us):", " ".join(f"{i}:{t[i]:.0f}" for i in sorted(slow)))
import torch  # noqa: E402

pr = torch.cuda.get_device_properties(0)
st = b.stats()
print(f"  device {pr.name} CUs {pr.multi_processor_count}; stats over the timed passes: "
      f"pre_gated {st['pre_gated'] / passes:.0f} post_gated {st['post_gated'] / passes:.0f} per pass")
