"""The sharded lastVisited merge (abnn.h abnn_shard_visits_delta / _merge,
DESIGN.md §7) on the CPU oracle's shard phases, in one process.

Unsharded, lastVisited[n] is the LAST value written (README §4: every visit
writes the pass's clock; the host may write any value).  A plain MAX over the
shards' copies is wrong after a renormalisation (a stamp from before it
outvotes a later, smaller one) and after a host write ahead of the clock;
the merge of marked visits is exact.  The gloo world-2/3 runs of the same
rule are in tests/test_sharded_gloo.py, the GPU's in
tests/test_gpu_parity.py::test_virtual_shards_visits_merge."""
import numpy as np
import pytest

from shard_helpers import merge_visits_local, oracle_shard_pass, shard_pass_merging

N_HIDDEN, N_SYN, PASSES = 20_000, 300_000, 9


def _shards(world, O, **kw):
    from abnn_amd.shard import global_events, shard_ranges

    ge = global_events(N_SYN, N_SYN, world)
    out = []
    for lo, hi in shard_ranges(N_SYN, world):
        ob = O.OracleBrain(256, 256, N_HIDDEN, hi - lo, N_SYN, syn_offset=lo, global_events=ge, **kw)
        ob.build_random_graph(seed=11, nthreads=2)
        ob.set_auto_stimulus(0, 256)
        out.append(ob)
    return out


def _unsharded(O, **kw):
    ref = O.OracleBrain(256, 256, N_HIDDEN, N_SYN, N_SYN, **kw)
    ref.build_random_graph(seed=11, nthreads=2)
    ref.set_auto_stimulus(0, 256)
    return ref


@pytest.mark.parametrize("world", [2, 3])
def test_marked_merge_equals_unsharded_where_plain_max_does_not(world):
    from oracle import oracle as O

    kw = dict(track_visits=1, renorm_thresh=2)  # clock 0 1 2 3 | 0 1 2 3 | 0
    ahead = (600, 8400, 3)  # before pass 4: lastVisited[600:9000] = clock + 3 (= pass 7's clock)
    ref = _unsharded(O, **kw)
    shards = _shards(world, O, **kw)
    plain = _shards(world, O, **kw)
    for k in range(PASSES):
        if k == 4:
            first, n, a = ahead
            for x in [ref, *shards, *plain]:
                x.set_last_visited(np.full(n, x.clock + a, np.uint64), first)
        ref.pass_serial()
        shard_pass_merging(shards, lambda: oracle_shard_pass(shards))
        oracle_shard_pass(plain)
    merge_visits_local(shards)
    assert ref.renormalisations() == 2
    for s in shards:
        assert np.array_equal(s.last_visited, ref.last_visited)
        assert np.array_equal(s.last_fired, ref.last_fired)
    # the old rule: all-reduce(MAX) of the whole arrays
    mx = np.maximum.reduce([p.last_visited for p in plain])
    assert not np.array_equal(mx, ref.last_visited)


def test_merge_without_track_visits_is_a_no_op():
    from oracle import oracle as O

    shards = _shards(2, O)
    for _ in range(3):
        shard_pass_merging(shards, lambda: oracle_shard_pass(shards))
    assert all(s.visit_mark is None for s in shards)
    merge_visits_local(shards)
    assert all(not s.last_visited.any() for s in shards)
