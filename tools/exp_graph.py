"""Pass time with and without hipGraph replay (ABNN_GRAPH), timing off,
config 3, one process per setting (the env var is read at create).  The
graph path was measured slower (profiles/r01_hipgraph_ab.txt) and removed
from the library; re-adding it is what this script would A/B again."""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROG = r'''
import sys, time; sys.path.insert(0, %r)
import abnn_amd
from abnn_amd import CONFIGS
wl = CONFIGS["c3"]
b = abnn_amd.Brain(wl.n_input, wl.n_output, wl.n_hidden, wl.n_syn, wl.events)
b.build_random_graph(1); b.set_auto_stimulus(0, 256)
b.encode_traversal(12); b.synchronize()
ts = []
for r in range(5):
    t0 = time.perf_counter(); b.encode_traversal(40); b.synchronize(); ts.append((time.perf_counter() - t0) / 40)
ts.sort(); print("RESULT", ts[2] * 1e3, b.checksum())
'''
res = {}
for rnd in range(2):
    for g in ("0", "1"):
        env = dict(os.environ, ABNN_GRAPH=g)
        r = subprocess.run([sys.executable, "-c", PROG % ROOT], capture_output=True, text=True, env=env, timeout=400)
        line = [l for l in r.stdout.splitlines() if l.startswith("RESULT")]
        if not line:
            print("FAILED", g, r.stderr[-800:]); sys.exit(1)
        ms, ck = line[0].split()[1:]
        res.setdefault(g, []).append((float(ms), ck))
for g, v in res.items():
    print(f"ABNN_GRAPH={g}: pass ms {[round(x[0], 4) for x in v]} checksum {v[0][1]}")
