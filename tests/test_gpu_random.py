"""GPU parity of random-edge mode (README §4; contract in include/abnn/abnn.h):
Philox picks, pass-start reads, highest-event-wins weight stores (k_claim),
track_visits, sharded picks -- HIP path vs the CPU oracle, bit-exact.  There is
no reference code for this mode, so the oracle (itself cross-checked against
an independent Python restatement in tests/test_oracle.py) is the only pin."""
import numpy as np
import pytest

from shard_helpers import GpuShards, oracle_shard_pass

pytestmark = pytest.mark.gpu


def _pair(n_hidden, n_syn, events, graph_seed=5, syn_offset=0, global_events=0, **params):
    import abnn_amd
    from oracle import oracle as O

    params.setdefault("mode", 1)
    params.setdefault("seed", 9)
    g = abnn_amd.Brain(256, 256, n_hidden, n_syn, events, syn_offset=syn_offset,
                       global_events=global_events, **params)
    g.build_random_graph(graph_seed)
    o = O.OracleBrain(256, 256, n_hidden, n_syn, events, syn_offset=syn_offset,
                      global_events=global_events, **params)
    o.build_random_graph(graph_seed, nthreads=16)
    g.set_auto_stimulus(0, 256)
    o.set_auto_stimulus(0, 256)
    return g, o


def _same(g, o, what=""):
    assert np.array_equal(g.download_synapses().view(np.uint32), o.syn.view(np.uint32)), f"synapses {what}"
    assert np.array_equal(g.last_fired(), o.last_fired), f"lastFired {what}"
    sg, so = g.scalars(), o.scalars()
    assert sg["clock"] == so["clock"] and sg["pass_index"] == so["pass_index"], what
    assert np.float32(sg["rbar"]) == np.float32(so["rbar"]), what


def test_random_collisions_every_pass(gpu):
    # 2000 synapses, 12000 picks per pass: ~6 visits per synapse, colliding updates every pass
    g, o = _pair(488, 2_000, 12_000)
    for k in range(16):
        if k == 7:
            g.set_reward(0.8)
            o.set_reward(0.8)
        g.encode_traversal(1)
        o.pass_serial()
        _same(g, o, f"pass {k}")
    assert g.stats() == o.stats()
    assert g.visited_events() == 12_000


def test_random_hidden_graph(gpu):
    g, o = _pair(20_000, 300_000, 250_000)
    for k in range(10):
        g.encode_traversal(1)
        o.pass_threaded(nthreads=16)
        _same(g, o, f"pass {k}")
    assert g.stats() == o.stats()


def test_random_c2_lite(gpu):
    g, o = _pair(99_488, 1_000_000, 1_500_000)
    for k in range(9):
        g.encode_traversal(1)
        o.pass_threaded(nthreads=16)
    _same(g, o)
    assert g.stats() == o.stats()


def test_random_track_visits(gpu):
    g, o = _pair(488, 5_000, 20_000, track_visits=1)
    for _ in range(6):
        g.encode_traversal(1)
        o.pass_serial()
    _same(g, o)
    assert np.array_equal(g.last_visited(), o.last_visited)


@pytest.mark.parametrize("over", [{"max_spikes": 0}, {"max_spikes": 1}, {"window_pre": 0},
                                  {"refractory": 0}])
def test_random_edge_parameters(gpu, over):
    g, o = _pair(488, 3_000, 10_000, **over)
    for _ in range(8):
        g.encode_traversal(1)
        o.pass_serial()
    _same(g, o, str(over))
    assert g.stats() == o.stats()


def test_random_virtual_shards_vs_oracle_shards(gpu):
    """Each shard picks within its own records with its own stream (key ^ syn_offset)."""
    import torch

    import abnn_amd
    from abnn_amd.shard import global_events, shard_ranges
    from oracle import oracle as O

    world, n_syn, events, passes = 3, 600_000, 200_000, 8
    ge = global_events(n_syn, events, world, 1)
    shards, obs = [], []
    for lo, hi in shard_ranges(n_syn, world):
        b = abnn_amd.Brain(256, 256, 30_000, hi - lo, events, syn_offset=lo, global_events=ge, mode=1, seed=3)
        b.build_random_graph(4)
        b.set_auto_stimulus(0, 256)
        shards.append(b)
        ob = O.OracleBrain(256, 256, 30_000, hi - lo, events, syn_offset=lo, global_events=ge, mode=1, seed=3)
        ob.build_random_graph(4, nthreads=16)
        ob.set_auto_stimulus(0, 256)
        obs.append(ob)
    gs = GpuShards(shards)
    for k in range(passes):
        gs.pass_()
        oracle_shard_pass(obs)
    torch.cuda.synchronize()
    for b, ob in zip(shards, obs):
        _same(b, ob, "shard")
