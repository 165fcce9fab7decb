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


@pytest.mark.gpu
def test_native_rccl_two_ranks_two_gpus(gpu):
    """The C-driven RCCL pass at world 2 (one GPU per rank, the in-place
    ncclAllGather with two records, rank_offset of rank 1): every rank's shard,
    lastFired, lastVisited and scalars equal the unsharded brain.  Needs two
    GPUs: skipped on a one-GPU box, so it runs wherever a node has them
    (UNVERIFIED on hardware until then: DESIGN.md §7)."""
    import abnn_amd

    if abnn_amd.device_count() < 2:
        pytest.skip("needs 2 GPUs (native RCCL at world 2)")
    n_syn = 2_000_000
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "helpers", "shard_worker.py"), str(n_syn), str(n_syn), "10", "native"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600,
                       env={**os.environ, "OMP_NUM_THREADS": "4"})
    assert r.returncode == 0, r.stderr[-3000:]
    assert "SHARDED_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.gpu
def test_native_rccl_shard_traverse_world1(gpu, monkeypatch):
    """The C-driven sharded pass (abnn_comm over RCCL, abnn_shard_traverse: gate,
    in-place ncclAllGather and apply/commit enqueued by the library, no Python
    per pass) at world 1 on the box's one GPU, with plasticity so the
    structural update's all-reduce of visited events runs: equal to the
    unsharded brain bit for bit."""
    import numpy as np
    import torch.distributed as dist

    import abnn_amd
    from abnn_amd.shard import ShardedBrain, TorchComm

    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        # track_visits with renormalisations after passes 5 and 11 (the
        # library merges lastVisited after each, over RCCL) and a host write
        # ahead of the clock before pass 7
        extra = dict(w_prune=0.105, p_new=0.35, w_init=0.5, compact_every=4, track_visits=1, renorm_thresh=4)
        n_syn, events, passes = 1_000_000, 1_000_000, 13
        sb = ShardedBrain(TorchComm(), 256, 256, 30_000, n_syn, events, device=0, capacity_factor=1.05,
                          native=True, **extra)
        ref = abnn_amd.Brain(256, 256, 30_000, n_syn, events, syn_capacity=int(n_syn * 1.05), **extra)
        for b in (sb.brain, ref):
            b.build_random_graph(4)
            b.set_auto_stimulus(0, 256)
            b.set_reward(0.25)
        sb.step(7)
        ref.encode_traversal(7)
        for b in (sb.brain, ref):
            b.set_last_visited(np.full(8400, b.scalars()["clock"] + 2, np.uint64), 600)
        sb.step(passes - 7)
        ref.encode_traversal(passes - 7)
        sb.sync_visits()
        ref.synchronize()
        assert sb.brain.renormalisations() == ref.renormalisations() == 2
        assert sb.brain.structural_updates() == ref.structural_updates() == 3
        assert np.array_equal(sb.brain.download_synapses().view(np.uint32), ref.download_synapses().view(np.uint32))
        assert np.array_equal(sb.brain.last_fired(), ref.last_fired())
        assert np.array_equal(sb.brain.last_visited(), ref.last_visited())
        assert sb.brain.scalars() == ref.scalars()
        assert sb.brain.stats() == ref.stats()
        sb.native.close()
    finally:
        dist.destroy_process_group()
