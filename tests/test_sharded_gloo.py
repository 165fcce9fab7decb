"""world_size-2 (and 3) multi-process test of the sharded pass on CPU over gloo.

Every rank runs the product's exchange logic (abnn_amd.shard.sharded_pass +
TorchComm + shard_ranges/global_events) with a CPU stand-in engine built on the
oracle's shard phases; the result must equal the unsharded serial C1 run
bit-for-bit.  The GPU engine plugs into the same sharded_pass (tests/test_gpu_*).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

N_HIDDEN, N_SYN, PASSES = 20_000, 300_000, 9


class CpuShardEngine:
    def __init__(self, ob):
        self.ob = ob

    def gate(self, xchg):
        self.ob.shard_gate(xchg.numpy())

    def apply(self, gathered, world, rank):
        self.ob.shard_apply(gathered.numpy(), world, rank)

    def commit(self, gathered, world):
        self.ob.shard_commit(gathered.numpy(), world)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, events, track):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch.distributed as dist
    from abnn_amd.shard import TorchComm, global_events, shard_ranges, sharded_pass
    from oracle import oracle as O

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = TorchComm()
        lo, hi = shard_ranges(N_SYN, world)[rank]
        ge = global_events(N_SYN, events, world)
        ob = O.OracleBrain(256, 256, N_HIDDEN, hi - lo, events, syn_offset=lo, global_events=ge,
                           track_visits=track)
        ob.build_random_graph(seed=11, nthreads=2)
        ob.set_auto_stimulus(0, 256)
        eng = CpuShardEngine(ob)
        words = ob.exchange_words()
        xchg = torch.zeros(words, dtype=torch.int32)
        gathered = torch.zeros(words * world, dtype=torch.int32)
        for k in range(PASSES):
            if k == 6:
                ob.set_reward(0.25)
            sharded_pass(eng, comm, xchg, gathered)
        if track:  # lazy lastVisited merge (all-reduce MAX)
            t = torch.from_numpy(ob.last_visited.view(np.int64).copy())
            comm.all_reduce_max(t)
            ob.last_visited[:] = t.numpy().view(np.uint64)

        # unsharded reference, computed independently on every rank
        ref = O.OracleBrain(256, 256, N_HIDDEN, N_SYN, events if world == 1 else N_SYN,
                            track_visits=track)
        ref.build_random_graph(seed=11, nthreads=2)
        ref.set_auto_stimulus(0, 256)
        for k in range(PASSES):
            if k == 6:
                ref.set_reward(0.25)
            ref.pass_serial()
        assert np.array_equal(ob.syn.view(np.uint32), ref.syn[lo:hi].view(np.uint32))
        assert np.array_equal(ob.last_fired, ref.last_fired)
        assert ob.clock == ref.clock
        assert np.float32(ob.s.rbar) == np.float32(ref.s.rbar)
        if track:
            assert np.array_equal(ob.last_visited, ref.last_visited)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,track", [(2, 0), (3, 0), (2, 1)])
def test_sharded_gloo_equals_unsharded(world, track):
    # events >= every shard's size: each shard sweeps its whole range, so the
    # rank-ordered union is the unsharded full sweep
    mp.spawn(_worker, args=(world, _free_port(), N_SYN, track), nprocs=world, join=True)


SP = dict(w_prune=0.105, p_new=0.35, w_init=0.5, compact_every=2)


def _shard_brains(world, events, extra, O, shard_ranges, ge, cap_factor):
    out = []
    for lo, hi in shard_ranges(N_SYN, world):
        ob = O.OracleBrain(256, 256, N_HIDDEN, hi - lo, events, syn_offset=lo, global_events=ge,
                           syn_capacity=int((hi - lo) * cap_factor), **extra)
        ob.build_random_graph(seed=11, nthreads=2)
        ob.set_auto_stimulus(0, 256)
        out.append(ob)
    return out


def _worker_modes(rank, world, port, events, extra):
    """Random-edge mode / structural plasticity: shards pick and grow within
    their own records, so the reference is the same shard phases run in one
    process (what the exchange must reproduce), not an unsharded run."""
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch.distributed as dist
    from abnn_amd.shard import TorchComm, global_events, shard_ranges, sharded_pass
    from oracle import oracle as O

    sys.path.insert(0, os.path.join(root, "tests"))
    from shard_helpers import oracle_shard_pass

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = TorchComm()
        ge = global_events(N_SYN, events, world, extra.get("mode", 0))
        cap = 1.1 if extra.get("p_new") else 1.0
        ob = _shard_brains(world, events, extra, O, shard_ranges, ge, cap)[rank]
        eng = CpuShardEngine(ob)
        words = ob.exchange_words()
        xchg = torch.zeros(words, dtype=torch.int32)
        gathered = torch.zeros(words * world, dtype=torch.int32)
        for k in range(PASSES):
            if k == 4:
                ob.set_reward(0.3)
            sharded_pass(eng, comm, xchg, gathered)

        ref = _shard_brains(world, events, extra, O, shard_ranges, ge, cap)
        for k in range(PASSES):
            if k == 4:
                for r in ref:
                    r.set_reward(0.3)
            oracle_shard_pass(ref)
        me = ref[rank]
        assert int(ob.s.dims.n_syn) == int(me.s.dims.n_syn)
        assert np.array_equal(ob.syn.view(np.uint32), me.syn.view(np.uint32))
        assert np.array_equal(ob.last_fired, me.last_fired)
        assert ob.scalars() == me.scalars() and ob.stats() == me.stats()
        if extra.get("p_new"):
            assert ob.stats()["pruned"] > 0 or ob.stats()["grown"] > 0
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("extra,events", [(dict(mode=1, seed=5), 120_000),
                                          (dict(SP, seed=5), N_SYN),
                                          (dict(SP, mode=1, seed=5), 120_000)],
                         ids=["random", "plasticity", "random+plasticity"])
def test_sharded_gloo_modes_equal_phase_sequence(extra, events):
    mp.spawn(_worker_modes, args=(2, _free_port(), events, extra), nprocs=2, join=True)
