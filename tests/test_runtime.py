"""Process-level integration: one HIP runtime whatever the import order."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROG = r'''
import sys; sys.path.insert(0, %r)
import abnn_amd
b = abnn_amd.Brain(256, 256, 488, 10_000, 100_000)
b.build_random_graph(1)
b.encode_traversal(4)
import torch
x = torch.ones(1024, device="cuda")
torch.cuda.synchronize()
maps = open("/proc/self/maps").read()
hips = {l.split()[-1] for l in maps.splitlines() if "libamdhip64" in l}
print("OK", len(hips), float(x.sum()))
''' % ROOT


@pytest.mark.gpu
def test_engine_then_torch_share_one_hip_runtime(gpu):
    r = subprocess.run([sys.executable, "-c", PROG], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.split()[:2] == ["OK", "1"], r.stdout
