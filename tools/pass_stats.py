"""Per-pass statistics and gate-kernel time at a config (GPU): shows how the
gate's cost follows the pass's dynamics (pre-gated entries, filter density)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import abnn_amd
from abnn_amd.configs import CONFIGS

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
b = abnn_amd.Brain(cfg.n_input, cfg.n_output, cfg.n_hidden, cfg.n_syn, cfg.events)
b.build_random_graph(1)
b.set_auto_stimulus(0, cfg.n_input)
b.encode_traversal(12)
b.synchronize()
b.enable_timing(True)
print("pass  gate_us  events  pre_gated  post_gated  updated  fired  recent")
for p in range(12):
    b.reset_stats()
    lf = b.last_fired()
    now = b.scalars()["clock"]
    recent = int(np.count_nonzero((now - lf.astype(np.int64)) <= b.params.window_pre))
    b.kernel_time()  # reset accumulator
    b.encode_traversal(1)
    b.synchronize()
    ms, n = b.kernel_time()
    s = b.stats()
    print(f"{p:4d} {ms * 1000 / max(n, 1):8.1f} {s['events']:9d} {s['pre_gated']:9d} {s['post_gated']:9d} "
          f"{s['updated']:8d} {s['fired']:6d} {recent:7d}")
