"""Multi-process sharded passes on the GPU: torchrun, 2 ranks sharing GPU 0,
gloo exchange (RCCL needs one GPU per rank); every rank checks its shard
against an unsharded GPU run (tests/helpers/shard_worker.py)."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_two_rank_sharded_brain_equals_unsharded(gpu):
    n_syn = 2_000_000
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "helpers", "shard_worker.py"), str(n_syn), str(n_syn), "10"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600,
                       env={**os.environ, "OMP_NUM_THREADS": "4"})
    assert r.returncode == 0, r.stderr[-3000:]
    assert "SHARDED_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
