"""Per-pass statistics and gate-kernel time at a config (GPU): shows how the
gate's cost follows the pass's dynamics (pre-gated entries, filter density).

usage: pass_stats.py [config] [first_pass] [n_passes]
Runs `first_pass` untimed passes, then prints one line per pass."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import abnn_amd
from abnn_amd.configs import CONFIGS

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
first = int(sys.argv[2]) if len(sys.argv) > 2 else 12
count = int(sys.argv[3]) if len(sys.argv) > 3 else 12
b = abnn_amd.Brain(cfg.n_input, cfg.n_output, cfg.n_hidden, cfg.n_syn, cfg.events)
b.build_random_graph(1)
b.set_auto_stimulus(0, cfg.n_input)
if first:
    b.encode_traversal(first)
b.synchronize()
b.enable_timing(True)
print("pass  gate_us  wall_us  events  pre_gated  post_gated  updated  fired  recent", flush=True)
for p in range(first, first + count):
    b.reset_stats()
    lf = b.last_fired()
    now = b.scalars()["clock"]
    recent = int(np.count_nonzero((now - lf.astype(np.int64)) <= b.params.window_pre))
    b.kernel_time()  # reset accumulator
    t0 = time.perf_counter()
    b.encode_traversal(1)
    b.synchronize()
    wall = (time.perf_counter() - t0) * 1e6
    ms, n = b.kernel_time()
    s = b.stats()
    print(f"{p:4d} {ms * 1000 / max(n, 1):8.1f} {wall:8.1f} {s['events']:9d} {s['pre_gated']:9d} "
          f"{s['post_gated']:9d} {s['updated']:8d} {s['fired']:6d} {recent:7d}", flush=True)
