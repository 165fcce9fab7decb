"""A/B the production gate kernel against ablation builds (tools/exp/*.so),
interleaved in separate processes on one GPU.  Results are timing-only: the
ablated builds do not produce correct traversals."""
import os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libs = {"prod": os.path.join(ROOT, "abnn_amd", "libabnn_hip.so")}
for f in sorted(os.listdir(os.path.join(ROOT, "tools", "exp"))):
    libs[f[len("libabnn_hip_"):-3]] = os.path.join(ROOT, "tools", "exp", f)
PROG = r'''
import sys, time; sys.path.insert(0, %r)
from abnn_amd import _lib
_lib.LIB_PATH = %r
import abnn_amd
from abnn_amd import CONFIGS
wl = CONFIGS["c3"]
b = abnn_amd.Brain(wl.n_input, wl.n_output, wl.n_hidden, wl.n_syn, wl.events)
b.build_random_graph(1); b.set_auto_stimulus(0, 256)
b.encode_traversal(10); b.synchronize(); b.enable_timing(True)
t0 = time.perf_counter(); b.encode_traversal(30); b.synchronize(); dt = time.perf_counter() - t0
ms, n = b.kernel_time()
print("RESULT", dt / 30 * 1e3, ms / n)
'''
res = {k: [] for k in libs}
for rnd in range(3):
    for k, lib in libs.items():
        r = subprocess.run([sys.executable, "-c", PROG % (ROOT, lib)], capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("RESULT")]
        if not line:
            print(k, "FAILED", r.stderr[-500:]); sys.exit(1)
        res[k].append(tuple(map(float, line[0].split()[1:])))
for k, v in res.items():
    v.sort(key=lambda x: x[1])
    print(f"{k:12s} gate median {v[1][1]:.4f} ms  pass median {sorted(x[0] for x in v)[1]:.4f} ms")
