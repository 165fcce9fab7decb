"""Parity at the benchmark's full size (config c3: 5,000,512 neurons, 1B
synapses, 150M events per pass) -- the HIP pass against the threaded C oracle,
bit-exact, after 80 passes from the freshly built graph (into the steady state).

Sizes the small parity tests never reach are exercised here: neuron ids above
2^18 (the pre-spike filter's block hash and rotation, engine.h / kernels.hip),
thousands of ranges and workgroups, the adaptive partition, the candidate lists
of dense ranges, the budget cut far inside the sweep.  The sweep touches only
the first E = 150M records, so the oracle holds exactly those (the generator is
per-record, bench.py cpu_baseline does the same): lastFired of every neuron,
the statistics, the scalars and all E records must match."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PASSES = 80


@pytest.mark.parametrize("env", [{}, {"ABNN_FUSED": "0"}, {"ABNN_SPEC": "2"}, {"ABNN_STATIC_RANGES": "1"}],
                         ids=["fused", "two-kernel", "spec-everywhere", "static-ranges"])
def test_c3_full_size_parity(gpu, monkeypatch, env):
    """The results may not depend on the partition (adaptive: timing-driven,
    so it differs from run to run and box to box), the path or speculation."""
    from abnn_amd import CONFIGS, Brain
    from oracle import oracle as O

    for k, v in env.items():
        monkeypatch.setenv(k, v)
    wl = CONFIGS["c3"]
    g = Brain(wl.n_input, wl.n_output, wl.n_hidden, wl.n_syn, wl.events)
    E = g.visited_events()
    o = O.OracleBrain(wl.n_input, wl.n_output, wl.n_hidden, E, wl.events)
    assert O.visited_events(wl.events, E) == E
    g.build_random_graph(1)
    o.build_random_graph(1, nthreads=16)
    g.set_auto_stimulus(0, wl.n_input)
    o.set_auto_stimulus(0, wl.n_input)
    g.encode_traversal(PASSES)
    o.pass_threaded(PASSES, nthreads=16)
    g.synchronize()

    sg, so = g.scalars(), o.scalars()
    assert sg["clock"] == so["clock"] and sg["pass_index"] == so["pass_index"]
    assert np.float32(sg["rbar"]) == np.float32(so["rbar"])
    assert g.stats() == o.stats()
    assert np.array_equal(g.last_fired(), o.last_fired)
    step = 10_000_000
    for first in range(0, E, step):
        n = min(step, E - first)
        assert np.array_equal(g.download_synapses(first, n).view(np.uint32),
                              o.syn[first:first + n].view(np.uint32)), f"records [{first}, {first + n})"


def test_c3_random_mode_full_size(gpu):
    """Random-edge mode (README §4; abnn.h) at config 3: the 1B-record graph,
    150M Philox picks per pass over all of it (the src32 mirror, the claim
    words, k_claim's highest-event-wins stores and the two-kernel path at
    full size), 12 passes from the fresh graph through the transient (passes
    3-5 gate every pick) into the steady state, with the reward changed
    mid-run.  GPU vs the threaded oracle holding the whole graph: every
    neuron's lastFired, the statistics, the scalars and the checksum of all
    1e9 records, plus bit-exact records over a sample of 10M-record windows."""
    from abnn_amd import CONFIGS, Brain
    from oracle import oracle as O

    wl = CONFIGS["c3"]
    g = Brain(wl.n_input, wl.n_output, wl.n_hidden, wl.n_syn, wl.events, mode=1, seed=9)
    o = O.OracleBrain(wl.n_input, wl.n_output, wl.n_hidden, wl.n_syn, wl.events, mode=1, seed=9)
    assert g.visited_events() == wl.events
    g.build_random_graph(1)
    o.build_random_graph(1, nthreads=16)
    for x in (g, o):
        x.set_auto_stimulus(0, wl.n_input)
    for k in range(12):
        if k == 7:
            g.set_reward(0.5)
            o.set_reward(0.5)
        g.encode_traversal(1)
        o.pass_threaded(1, nthreads=16)
    g.synchronize()
    sg, so = g.scalars(), o.scalars()
    assert sg["clock"] == so["clock"] == 12 and sg["pass_index"] == so["pass_index"]
    assert np.float32(sg["rbar"]) == np.float32(so["rbar"])
    st = g.stats()
    assert st == o.stats()
    assert st["fired"] > 2560 * 4 and st["updated"] > st["fired"]
    assert np.array_equal(g.last_fired(), o.last_fired)
    assert g.checksum() == o.checksum()
    step = 10_000_000
    for first in range(0, wl.n_syn, 97_000_000):
        assert np.array_equal(g.download_synapses(first, step).view(np.uint32),
                              o.syn[first:first + step].view(np.uint32)), f"records [{first}, {first + step})"


def test_c4_eight_virtual_shards_of_the_1b_graph(gpu):
    """Config 4's workload on one GPU: the 1B-synapse c3 graph in 8 contiguous
    shards of 125M records, 150M events per shard per pass (so every shard
    sweeps its whole shard), driven through the real shard entry points
    (abnn_shard_gate / apply / commit) around an in-process all-gather of the
    exchange records.  25 passes into the steady state; then every shard's
    records (position-sensitive checksums, which add up over shards, plus a
    10M-record slice of each), lastFired, the clock and rBar must equal an
    unsharded GPU full sweep (events = N_SYN), which in turn must equal the
    threaded oracle on the whole graph (BASELINE.json configs[3])."""
    import abnn_amd
    from abnn_amd import CONFIGS
    from abnn_amd.shard import global_events, shard_ranges
    from oracle import oracle as O
    from shard_helpers import GpuShards

    wl, world, passes = CONFIGS["c3"], 8, 25
    ge = global_events(wl.n_syn, wl.events, world)
    assert ge == wl.n_syn  # each shard's 150M-event sweep covers its 125M records
    shards = []
    for lo, hi in shard_ranges(wl.n_syn, world):
        b = abnn_amd.Brain(wl.n_input, wl.n_output, wl.n_hidden, hi - lo, wl.events, syn_offset=lo, global_events=ge)
        b.build_random_graph(1)
        b.set_auto_stimulus(0, wl.n_input)
        assert b.visited_events() == hi - lo
        shards.append(b)
    vs = GpuShards(shards)
    for _ in range(passes):
        vs.pass_()
    full = abnn_amd.Brain(wl.n_input, wl.n_output, wl.n_hidden, wl.n_syn, wl.n_syn)
    full.build_random_graph(1)
    full.set_auto_stimulus(0, wl.n_input)
    full.encode_traversal(passes)
    full.synchronize()

    sf = full.scalars()
    lf = full.last_fired()
    assert sf["clock"] == passes
    csum = 0
    for r, (b, (lo, hi)) in enumerate(zip(shards, shard_ranges(wl.n_syn, world))):
        s = b.scalars()
        assert (s["clock"], s["pass_index"]) == (sf["clock"], sf["pass_index"]), r
        assert np.float32(s["rbar"]) == np.float32(sf["rbar"]), r
        assert np.array_equal(b.last_fired(), lf), r
        csum = (csum + b.checksum()) & (2**64 - 1)
        n = 10_000_000
        first = (hi - lo) - n if r % 2 else 0
        assert np.array_equal(b.download_synapses(first, n).view(np.uint32),
                              full.download_synapses(lo + first, n).view(np.uint32)), r
    assert csum == full.checksum()
    st = [b.stats() for b in shards]
    fs = full.stats()
    assert sum(x["events"] for x in st) == fs["events"] == passes * wl.n_syn
    assert sum(x["fired"] for x in st) == fs["fired"]
    assert sum(x["updated"] for x in st) == fs["updated"]
    del shards, vs

    o = O.OracleBrain(wl.n_input, wl.n_output, wl.n_hidden, wl.n_syn, wl.n_syn)
    o.build_random_graph(1, nthreads=16)
    o.set_auto_stimulus(0, wl.n_input)
    o.pass_threaded(passes, nthreads=16)
    assert o.checksum() == full.checksum()
    assert np.array_equal(o.last_fired, lf)
    assert o.stats() == fs
    assert np.float32(o.s.rbar) == np.float32(sf["rbar"]) and o.clock == sf["clock"]


def test_c4_random_mode_eight_virtual_shards(gpu):
    """Config 4's workload in random-edge mode (150M
    picks per GPU per pass; README §4): the 1B-record graph in 8 shards of
    125M records, each shard picking 150M records of its own per pass (its own
    Philox stream, keyed by syn_offset), through the real shard entry points
    around an in-process all-gather, 6 passes from the fresh graph through
    the all-gated transient (passes 3-5 gate every pick), reward changed
    mid-run.  Against the oracle's shard phases on the same 8 shards (run in
    parallel threads): every shard's checksum over its 125M records, a 10M-
    record slice of each, lastFired, statistics and scalars."""
    from concurrent.futures import ThreadPoolExecutor

    import abnn_amd
    from abnn_amd import CONFIGS
    from abnn_amd.shard import global_events, shard_ranges
    from oracle import oracle as O
    from shard_helpers import GpuShards

    wl, world, passes = CONFIGS["c3"], 8, 6
    kw = dict(mode=1, seed=9)
    ge = global_events(wl.n_syn, wl.events, world, 1)
    assert ge == world * wl.events
    shards, obs = [], []
    for lo, hi in shard_ranges(wl.n_syn, world):
        b = abnn_amd.Brain(wl.n_input, wl.n_output, wl.n_hidden, hi - lo, wl.events, syn_offset=lo,
                           global_events=ge, **kw)
        b.build_random_graph(1)
        b.set_auto_stimulus(0, wl.n_input)
        assert b.visited_events() == wl.events
        shards.append(b)
    pool = ThreadPoolExecutor(world)

    def make(r):
        lo, hi = shard_ranges(wl.n_syn, world)[r]
        ob = O.OracleBrain(wl.n_input, wl.n_output, wl.n_hidden, hi - lo, wl.events, syn_offset=lo,
                           global_events=ge, **kw)
        ob.build_random_graph(1, nthreads=2)
        ob.set_auto_stimulus(0, wl.n_input)
        return ob

    obs = list(pool.map(make, range(world)))
    vs = GpuShards(shards)
    words = obs[0].exchange_words()
    gathered = np.zeros(world * words, dtype=np.int32)
    for k in range(passes):
        if k == 4:
            for x in (*shards, *obs):
                x.set_reward(0.5)
        vs.pass_()
        # the oracle's shard phases, the gates (150M picks each) in parallel
        list(pool.map(lambda r: obs[r].shard_gate(gathered[r * words:(r + 1) * words]), range(world)))
        list(pool.map(lambda r: obs[r].shard_apply(gathered, world, r), range(world)))
        for ob in obs:
            ob.shard_commit(gathered, world)
    for r, (b, ob) in enumerate(zip(shards, obs)):
        sg, so = b.scalars(), ob.scalars()
        assert sg["clock"] == so["clock"] == passes and sg["pass_index"] == so["pass_index"], r
        assert np.float32(sg["rbar"]) == np.float32(so["rbar"]), r
        assert b.stats() == ob.stats(), r
        assert np.array_equal(b.last_fired(), ob.last_fired), r
        assert b.checksum() == ob.checksum(), r
        n = 10_000_000
        first = b.n_syn() - n if r % 2 else 0
        assert np.array_equal(b.download_synapses(first, n).view(np.uint32),
                              ob.syn[first:first + n].view(np.uint32)), r
    st = [b.stats() for b in shards]
    assert sum(x["fired"] for x in st) >= 2560 * 3 and sum(x["updated"] for x in st) > sum(x["fired"] for x in st)


def test_c5_4b_records_plasticity(gpu):
    """Config 5's size on one GPU: 4e9 records (44 GB of packed records; the
    structural update works in place), sweep mode, reward 0.25, pruning
    and synaptogenesis with a structural update every 10 passes (two inside
    the test).  Every pass: at most max_spikes spikes, one clock tick, n_syn =
    n_syn(before) - pruned + grown across updates, no tombstone left in the
    swept window after an update.  The threaded oracle holds the graph's
    first E + 4M records and its LAST 6M (the update's removal fills the
    window's tombstones with the array's last live records and ends the array
    before them: abnn.h), so at the end the GPU's whole array is pinned: the head and the
    tail (grown records included) bit-exact, the untouched middle by the
    whole-array checksum (the fresh graph's, less the head's and tail's)."""
    import abnn_amd
    from oracle import oracle as O

    n_in, n_out, n_hid, n_syn, events = 256, 256, 5_000_000, 4_000_000_000, 150_000_000
    n_nrn = n_in + n_out + n_hid
    extra = dict(w_prune=0.105, p_new=0.25, w_init=0.5, compact_every=10)
    grow = 1_000_000
    g = abnn_amd.Brain(n_in, n_out, n_hid, n_syn, events, syn_capacity=n_syn + grow, **extra)
    E = g.visited_events()
    slack, K = 4_000_000, 6_000_000
    H = E + slack
    head = O.gen_synapses(0, H, n_in, n_out, n_nrn, 1, 16)
    tail = O.gen_synapses(n_syn - K, K, n_in, n_out, n_nrn, 1, 16)
    mid = n_syn - K - H
    o = O.OracleBrain(n_in, n_out, n_hid, H + K, events, syn_capacity=H + K + grow, **extra)
    o.set_synapses(np.concatenate([head, tail]))
    g.build_random_graph(1)
    M = (1 << 64) - 1
    mid_ck = (g.checksum() - O.checksum(head, 0) - O.checksum(tail, n_syn - K)) & M  # the untouched middle
    del head, tail
    for x in (g, o):
        x.set_auto_stimulus(0, n_in)
        x.set_reward(0.25)
    prev = g.stats()
    n_prev = g.n_syn()
    pruned_since = 0
    for p in range(25):
        g.encode_traversal(1)
        st = g.stats()
        assert st["passes"] == p + 1 and g.scalars()["clock"] == p + 1
        assert st["fired"] - prev["fired"] <= 2560
        pruned_since += st["pruned"] - prev["pruned"]
        if (p + 1) % extra["compact_every"] == 0:
            assert g.structural_updates() == (p + 1) // extra["compact_every"]
            assert g.n_syn() == n_prev - pruned_since + (st["grown"] - prev["grown"])
            w = g.download_synapses(0, E)
            assert not np.any(w["src"] == 0xFFFFFFFF)  # compacted: no tombstone in the window
            n_prev, pruned_since = g.n_syn(), 0
        else:
            assert g.n_syn() == n_prev and st["grown"] == prev["grown"]
        prev = st
    assert g.structural_updates() == 2 and st["pruned"] > 0 and st["grown"] > 0
    o.pass_threaded(25, nthreads=16)
    assert st["pruned"] <= slack and st["pruned"] <= K
    so = o.stats()
    assert so == st
    assert np.array_equal(g.last_fired(), o.last_fired)
    sg = g.scalars()
    assert sg["clock"] == o.clock and np.float32(sg["rbar"]) == np.float32(o.s.rbar)
    # the whole array: GPU = head ++ middle (untouched) ++ rest, oracle = head ++ rest
    osyn = o.syn
    assert g.n_syn() == osyn.shape[0] + mid
    step = 10_000_000
    for first in range(0, H, step):
        n = min(step, H - first)
        assert np.array_equal(g.download_synapses(first, n).view(np.uint32),
                              osyn[first:first + n].view(np.uint32)), f"records [{first}, {first + n})"
    rest = osyn[H:]
    assert np.array_equal(g.download_synapses(H + mid, rest.shape[0]).view(np.uint32), rest.view(np.uint32))
    assert g.checksum() == (O.checksum(osyn[:H], 0) + mid_ck + O.checksum(rest, H + mid)) & M
