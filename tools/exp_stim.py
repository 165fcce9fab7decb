"""Experiment: gate-kernel time at config 3 with and without the input stimulus
(the dense input->output block is fully pre-gated every pass when inputs fire)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import abnn_amd
from abnn_amd import CONFIGS
wl = CONFIGS["c3"]
b = abnn_amd.Brain(wl.n_input, wl.n_output, wl.n_hidden, wl.n_syn, wl.events)
b.build_random_graph(1)
for stim in (256, 0, 256):
    b.set_auto_stimulus(0, stim)
    b.encode_traversal(10)
    b.synchronize()
    b.reset_stats(); b.enable_timing(True)
    t0 = time.perf_counter(); b.encode_traversal(30); b.synchronize(); dt = time.perf_counter() - t0
    ms, n = b.kernel_time(); st = b.stats()
    print(f"stim={stim:3d} pass {dt/30*1e3:.4f} ms gate {ms/n:.4f} ms  g1/pass {st['pre_gated']/30:.0f} fired/pass {st['fired']/30:.0f}", flush=True)
