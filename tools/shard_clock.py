#!/usr/bin/env python3
"""Per-workgroup timeline of k_shard_walk (the sharded pass's second launch) at
one GPU: the sharded pass at world 1 (abnn_shard_traverse over RCCL), then the
last pass's checkpoints (us after the earliest workgroup entry): entry,
scalars + range summary, range walk done, stamps issued, barrier (stores
drained), ticket returned.  usage: python tools/shard_clock.py [passes]"""
import ctypes
import os
import socket
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch.distributed as dist  # noqa: E402

from abnn_amd import CONFIGS  # noqa: E402
from abnn_amd.shard import ShardedBrain, TorchComm  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
with socket.socket() as so:
    so.bind(("127.0.0.1", 0))
    os.environ.setdefault("MASTER_PORT", str(so.getsockname()[1]))
dist.init_process_group("gloo", rank=0, world_size=1)
wl = CONFIGS[os.environ.get("CFG", "c3")]
sb = ShardedBrain(TorchComm(), wl.n_input, wl.n_output, wl.n_hidden, wl.n_syn, wl.events, device=0, native=True)
b = sb.brain
b.build_random_graph(1)
b.set_auto_stimulus(0, wl.n_input)
passes = int(sys.argv[1]) if len(sys.argv) > 1 else 100
sb.step(passes)
b.synchronize()
f = b._lib.abnn_debug_apply_clock
f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
f.restype = ctypes.c_int
buf = np.zeros(8 * 256, dtype=np.uint64)
assert f(b._h, buf.ctypes.data, buf.size) == 0
w = buf.reshape(-1, 8).astype(np.int64)
w = w[w[:, 0] > 0]
t0 = w[:, 0].min()
q = lambda x: " ".join(f"{v:6.2f}" for v in np.percentile(x, [0, 10, 50, 90, 100]))  # noqa: E731
for i, n in enumerate(["entry", "scalars+summary", "range walk", "stamps issued", "barrier", "ticket"]):
    print(f"{n:16s} {q((w[:, i] - t0) * 1e-2)}")
last = np.flatnonzero(w[:, 6] == 1)
if len(last):
    print("last workgroup:", " ".join(f"{(w[last[0], i] - t0) * 1e-2:.2f}" for i in range(6)))
sb.native.close()
dist.destroy_process_group()
