"""The C-driven sharded pass (abnn_shard_traverse: gate, all-gather, walk,
commit, the lastVisited merge and the structural update's all-reduce, all
enqueued by the library) at world 2, 3 and 8 on ONE GPU, over the in-process
communicator group (abnn_comm_group: one host thread per rank, the
collectives as device copies and a reduction kernel between host barriers --
SURVEY §4 item 4's fake communicator behind the same interface as RCCL).
This is the path `bench.py --gpus N` runs under RCCL; here every piece of it
except the RCCL calls themselves runs at world > 1: rank_offset > 0, the
in-place gather layout with several records, merge_visits and the
visited-events all-reduce."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _on_every_rank(fns):
    """Run fns[r]() on one thread per rank (the collectives need them all at
    once); re-raise the first failure after every thread has ended."""
    errs = [None] * len(fns)

    def run(r):
        try:
            fns[r]()
        except BaseException as e:  # noqa: BLE001 -- reported below
            errs[r] = e

    ts = [threading.Thread(target=run, args=(r,)) for r in range(len(fns))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=600)
    assert not any(t.is_alive() for t in ts), "a rank did not finish"
    for e in errs:
        if e is not None:
            raise e


def _shards(world, n_syn, events, nh, **kw):
    from abnn_amd.shard import LocalGroup, ShardedBrain

    g = LocalGroup(world)
    sbs = [ShardedBrain(g.comm(r, 0), 256, 256, nh, n_syn, events, device=0, **kw) for r in range(world)]
    return g, sbs


@pytest.mark.parametrize("world,max_spikes", [(2, 2560), (3, 20_000), (8, 10**8)])
def test_local_group_shard_traverse_equals_unsharded(gpu, world, max_spikes):
    """World 2 / 3 / 8 on one GPU against the unsharded brain, bit for bit:
    every record (the shards concatenated), lastFired, lastVisited (merged
    after each of two renormalisations, and on demand at the end), clock, rBar,
    pass index, renormalisations and the statistics.  The budget is the
    reference's at world 2 (its cut inside rank 0 or 1), 20,000 at world 3 and
    unbounded at world 8, so higher ranks' events fall below the cut and walk
    from rank_offset > 0.  A host write of lastVisited ahead of the clock
    before pass 7 (on every rank) must lose to later visits only."""
    import torch

    import abnn_amd

    n_syn, nh, passes = 2_000_000, 30_000, 13
    kw = dict(track_visits=1, renorm_thresh=4, max_spikes=max_spikes)
    g, sbs = _shards(world, n_syn, n_syn, nh, **kw)
    ref = abnn_amd.Brain(256, 256, nh, n_syn, n_syn, **kw)
    for b in [ref] + [sb.brain for sb in sbs]:
        b.build_random_graph(4)
        b.set_auto_stimulus(0, 256)
        b.set_reward(0.25)
    try:
        _on_every_rank([lambda sb=sb: sb.step(7) for sb in sbs])
        ref.encode_traversal(7)
        torch.cuda.synchronize()
        for b in [ref] + [sb.brain for sb in sbs]:
            b.set_last_visited(np.full(8400, b.scalars()["clock"] + 2, np.uint64), 600)
            b.set_reward(-0.5)
        _on_every_rank([lambda sb=sb: sb.step(passes - 7) for sb in sbs])
        ref.encode_traversal(passes - 7)
        _on_every_rank([lambda sb=sb: sb.sync_visits() for sb in sbs])
        ref.synchronize()
        assert ref.renormalisations() == 2
        whole = ref.download_synapses().view(np.uint32)
        lf, lv, sc = ref.last_fired(), ref.last_visited(), ref.scalars()
        for sb in sbs:
            b = sb.brain
            assert b.renormalisations() == 2, sb.rank
            assert np.array_equal(b.download_synapses().view(np.uint32),
                                  whole.reshape(-1, 4)[sb.lo:sb.hi].reshape(-1)), f"rank {sb.rank} records"
            assert np.array_equal(b.last_fired(), lf), f"rank {sb.rank} lastFired"
            assert np.array_equal(b.last_visited(), lv), f"rank {sb.rank} lastVisited"
            assert b.scalars() == sc, f"rank {sb.rank} scalars"
        st = [sb.brain.stats() for sb in sbs]
        fs = ref.stats()
        for k in ("pre_gated", "post_gated", "updated", "fired", "events"):
            assert sum(x[k] for x in st) == fs[k], k
        assert fs["fired"] > 0 and fs["updated"] > 0
        if world > 2:  # the budget reached past rank 0: some higher rank updated events
            assert any(x["updated"] for x in st[1:])
    finally:
        for sb in sbs:
            sb.brain.close()
        g.close()


@pytest.mark.parametrize("world", [2, 3])
def test_local_group_plasticity_vs_oracle_shards(gpu, world):
    """Structural plasticity on the C-driven path at world 2 / 3 (pruning,
    synaptogenesis, a structural update every 4 passes on every rank, then
    the all-reduce of the shards' visited events), with track_visits and
    renormalisations: every shard equals the oracle's shard phases (the
    reference restatement, tests/shard_helpers.py) -- records, record count,
    lastFired, merged lastVisited, scalars and per-shard statistics."""
    import torch

    from abnn_amd.shard import global_events, shard_ranges
    from oracle import oracle as O
    from shard_helpers import merge_visits_local, oracle_shard_pass

    n_syn, events, nh, passes = 240_000, 240_000, 3_000, 14
    kw = dict(w_prune=0.105, p_new=0.35, w_init=0.5, compact_every=4, track_visits=1, renorm_thresh=5)
    g, sbs = _shards(world, n_syn, events, nh, capacity_factor=1.1, **kw)
    ge = global_events(n_syn, events, world)
    obs = [O.OracleBrain(256, 256, nh, hi - lo, events, syn_offset=lo, global_events=ge,
                         syn_capacity=int((hi - lo) * 1.1), **kw) for lo, hi in shard_ranges(n_syn, world)]
    for x in obs + [sb.brain for sb in sbs]:
        x.build_random_graph(7)
        x.set_auto_stimulus(0, 256)
        x.set_reward(0.25)
    try:
        _on_every_rank([lambda sb=sb: sb.step(passes) for sb in sbs])
        for _ in range(passes):
            before = obs[0].renormalisations()
            oracle_shard_pass(obs)
            if obs[0].renormalisations() != before:
                merge_visits_local(obs)
        _on_every_rank([lambda sb=sb: sb.sync_visits() for sb in sbs])
        merge_visits_local(obs)
        torch.cuda.synchronize()
        assert obs[0].renormalisations() >= 2
        assert sbs[0].brain.structural_updates() == passes // 4
        for sb, o in zip(sbs, obs):
            b = sb.brain
            assert b.n_syn() == o.syn.shape[0], sb.rank
            assert np.array_equal(b.download_synapses().view(np.uint32), o.syn.view(np.uint32)), sb.rank
            assert np.array_equal(b.last_fired(), o.last_fired), sb.rank
            assert np.array_equal(b.last_visited(), o.last_visited), sb.rank
            s, os_ = b.scalars(), o.scalars()
            assert (s["clock"], s["pass_index"]) == (os_["clock"], os_["pass_index"]), sb.rank
            assert np.float32(s["rbar"]) == np.float32(os_["rbar"]), sb.rank
            assert b.stats() == o.stats(), sb.rank
        assert sum(o.stats()["pruned"] for o in obs) > 0 and sum(o.stats()["grown"] for o in obs) > 0
    finally:
        for sb in sbs:
            sb.brain.close()
        g.close()


def test_local_group_failed_rank_breaks_the_group(gpu):
    """A rank that fails before its collective (here: a pass refused because
    its records were invalidated) breaks the group: the other rank's pass
    returns an error instead of waiting for it forever."""
    from abnn_amd import _lib

    g, sbs = _shards(2, 200_000, 200_000, 3_000)
    try:
        for sb in sbs:
            sb.brain.build_random_graph(1)
        errs = []

        def rank0():
            try:
                sbs[0].brain.close()  # rank 0's handle is gone: its call fails at once
                _lib.call("abnn_shard_traverse", None, sbs[0].native.handle, 1, None)
            except _lib.AbnnError as e:
                errs.append(("r0", e))

        def rank1():
            try:
                sbs[1].step(1)
            except _lib.AbnnError as e:
                errs.append(("r1", e))

        _on_every_rank([rank0, rank1])
        assert {r for r, _ in errs} == {"r0", "r1"}, errs
    finally:
        for sb in sbs:
            sb.brain.close()
        g.close()
