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

    def tracks_visits(self):
        return bool(self.ob.p.track_visits)

    def renormalisations(self):
        return self.ob.renormalisations()

    def visits_delta(self):
        return torch.from_numpy(self.ob.visits_delta().copy())

    def visits_merge(self, reduced):
        self.ob.visits_merge(reduced.numpy())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# host write of lastVisited ahead of the clock: (before pass, (first neuron,
# count), value - pass-start clock) -- the same on every rank, as the neuron
# state is replicated.  With renorm_thresh 2 the clock runs 0 1 2 3 | 0 1 2 3
# | 0, so the written value 3 is also what pass 7's visits write
AHEAD = (4, (600, 8400), 3)


def _worker(rank, world, port, events, track, renorm):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch.distributed as dist
    from abnn_amd.shard import TorchComm, global_events, merge_visits, shard_ranges, sharded_pass
    from oracle import oracle as O

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    extra = dict(renorm_thresh=renorm) if renorm else {}
    try:
        comm = TorchComm()
        lo, hi = shard_ranges(N_SYN, world)[rank]
        ge = global_events(N_SYN, events, world)
        ob = O.OracleBrain(256, 256, N_HIDDEN, hi - lo, events, syn_offset=lo, global_events=ge,
                           track_visits=track, **extra)
        ob.build_random_graph(seed=11, nthreads=2)
        ob.set_auto_stimulus(0, 256)
        eng = CpuShardEngine(ob)
        words = ob.exchange_words()
        xchg = torch.zeros(words, dtype=torch.int32)
        gathered = torch.zeros(words * world, dtype=torch.int32)

        def host_write(x):  # abnn_set_last_visited of a contiguous range
            _, (first, n), ahead = AHEAD
            x.set_last_visited(np.full(n, x.clock + ahead, np.uint64), first)

        for k in range(PASSES):
            if k == 6:
                ob.set_reward(0.25)
            if track and k == AHEAD[0]:
                host_write(ob)
            sharded_pass(eng, comm, xchg, gathered)
        merge_visits(eng, comm)  # the lazy merge before lastVisited is read

        # unsharded reference, computed independently on every rank
        ref = O.OracleBrain(256, 256, N_HIDDEN, N_SYN, events if world == 1 else N_SYN,
                            track_visits=track, **extra)
        ref.build_random_graph(seed=11, nthreads=2)
        ref.set_auto_stimulus(0, 256)
        for k in range(PASSES):
            if k == 6:
                ref.set_reward(0.25)
            if track and k == AHEAD[0]:
                host_write(ref)
            ref.pass_serial()
        if renorm:
            assert ref.renormalisations() >= 2 and ob.renormalisations() == ref.renormalisations()
        assert np.array_equal(ob.syn.view(np.uint32), ref.syn[lo:hi].view(np.uint32))
        assert np.array_equal(ob.last_fired, ref.last_fired)
        assert ob.clock == ref.clock
        assert np.float32(ob.s.rbar) == np.float32(ref.s.rbar)
        if track:
            assert np.array_equal(ob.last_visited, ref.last_visited)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,track,renorm", [(2, 0, 0), (3, 0, 0), (2, 1, 0), (2, 1, 2), (3, 1, 2)])
def test_sharded_gloo_equals_unsharded(world, track, renorm):
    # events >= every shard's size: each shard sweeps its whole range, so the
    # rank-ordered union is the unsharded full sweep.  track + renorm: the
    # lastVisited merge across renormalisations (the clock goes back to 0
    # after passes 3 and 7) and a host write ahead of the clock
    mp.spawn(_worker, args=(world, _free_port(), N_SYN, track, renorm), nprocs=world, join=True)


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
