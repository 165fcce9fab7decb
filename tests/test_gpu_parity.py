"""GPU parity: the HIP path (through the C-ABI) vs the CPU oracle, bit-exact.

Weights: bit-exact fp32 (both sides round every operation, -ffp-contract=off).
Timestamps, clock, spike counts: bit-exact integers.  rBar: bit-exact fp32.
(The oracle itself is "parity unpinned" against the Metal reference: DESIGN.md §3.)
"""
import os

import numpy as np
import pytest

from shard_helpers import GpuShards, oracle_shard_pass

pytestmark = pytest.mark.gpu


def _pair(n_hidden, n_syn, events, seed=1, stim=True, syn_offset=0, global_events=0, **params):
    import abnn_amd
    from oracle import oracle as O

    g = abnn_amd.Brain(256, 256, n_hidden, n_syn, events, syn_offset=syn_offset,
                       global_events=global_events, **params)
    g.build_random_graph(seed)
    o = O.OracleBrain(256, 256, n_hidden, n_syn, events, syn_offset=syn_offset,
                      global_events=global_events, **params)
    o.build_random_graph(seed, nthreads=16)
    if stim:
        g.set_auto_stimulus(0, 256)
        o.set_auto_stimulus(0, 256)
    return g, o


def _assert_same(g, o, what=""):
    syn = g.download_synapses()
    assert np.array_equal(syn.view(np.uint32), o.syn.view(np.uint32)), f"synapses differ {what}"
    assert np.array_equal(g.last_fired(), o.last_fired), f"lastFired differs {what}"
    sg, so = g.scalars(), o.scalars()
    assert sg["clock"] == so["clock"], what
    assert np.float32(sg["rbar"]) == np.float32(so["rbar"]), what


def test_generator_parity(gpu):
    g, o = _pair(99_488, 3_000_000, 1000)
    assert g.checksum() == o.checksum()
    assert np.array_equal(g.download_synapses().view(np.uint32), o.syn.view(np.uint32))


def test_config1_every_pass(gpu):
    # BASELINE configs[0]: 1k neurons, 10k synapses, 100k events (10k visits)
    g, o = _pair(488, 10_000, 100_000)
    for k in range(64):
        if k == 20:
            g.set_reward(1.0)
            o.set_reward(1.0)
        g.encode_traversal(1)
        o.pass_serial()
        _assert_same(g, o, f"pass {k}")
    assert g.stats() == o.stats()


def test_wave_clock_only_on_request(gpu):
    """The per-wave diagnostic timeline (abnn_debug.h) is recorded only after
    abnn_debug_set_wave_clock(b, 1) -- its stores cost 1.6 us per fused pass
    (profiles/r06l_ab_wave_clock_stores.txt) -- and recording it changes no
    result: the pass with it on is still bit-exact against the oracle."""
    import ctypes

    g, o = _pair(99_488, 1_000_000, 1_000_000)
    f = g._lib.abnn_debug_wave_clock
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    buf = np.zeros(16 * 4096, dtype=np.uint64)
    for k in range(4):
        g.encode_traversal(1)
        o.pass_threaded(nthreads=16)
    assert f(g._h, buf.ctypes.data, buf.size) == 0
    assert not buf.any(), "wave clocks recorded while off"
    assert g._lib.abnn_debug_set_wave_clock(g._h, 1) == 0
    for k in range(4):
        g.encode_traversal(1)
        o.pass_threaded(nthreads=16)
        _assert_same(g, o, f"clocks on, pass {k}")
    assert f(g._h, buf.ctypes.data, buf.size) == 0
    w = buf.reshape(-1, 16)
    assert (w[:, 0] > 0).any() and (w[:, 1] >= w[:, 0]).all(), "stream start / end not recorded"
    assert g.stats() == o.stats()


def test_c2_lite_every_pass(gpu):
    # 100k neurons, 1M synapses: all-gated passes 3-5, then the budget-saturated steady state
    g, o = _pair(99_488, 1_000_000, 1_000_000)
    for k in range(12):
        g.encode_traversal(1)
        o.pass_threaded(nthreads=16)
        _assert_same(g, o, f"pass {k}")
    assert g.stats() == o.stats()


def test_config2_full_state(gpu):
    # BASELINE configs[1]: 100k neurons, 10M synapses, 10M events per pass
    g, o = _pair(99_488, 10_000_000, 10_000_000)
    for k in range(10):
        if k == 7:
            g.set_reward(-0.25)
            o.set_reward(-0.25)
        g.encode_traversal(1)
        o.pass_threaded(nthreads=16)
        if k in (3, 6, 9):
            _assert_same(g, o, f"pass {k}")
    assert g.stats() == o.stats()


@pytest.mark.parametrize("over", [
    dict(max_spikes=1), dict(max_spikes=0), dict(max_spikes=200_000),
    dict(refractory=0, window_pre=0), dict(refractory=6, window_pre=2), dict(refractory=5, window_pre=5),
    dict(events=777_777), dict(events=3_000_000),
    dict(events=100), dict(renorm_thresh=5), dict(track_visits=1),
    dict(a_ltp=0.5, a_ltd=0.3, eta_home=1e-3, base_scale=3.0),
])
def test_edge_cases(gpu, over):
    over = dict(over)
    events = over.pop("events", 1_500_000)
    g, o = _pair(50_000, 2_000_000, events, seed=5, **over)
    for k in range(14):
        if k == 9:
            g.set_reward(0.5)
            o.set_reward(0.5)
        g.encode_traversal(1)
        o.pass_threaded(nthreads=16)
    _assert_same(g, o, str(over))
    if over.get("track_visits"):
        assert np.array_equal(g.last_visited(), o.last_visited)
    if over.get("renorm_thresh"):
        assert g.scalars()["clock"] < 8
    assert g.stats() == o.stats()


@pytest.mark.parametrize("env", [{"ABNN_FUSED": "0"}, {"ABNN_SPEC": "2"}, {"ABNN_SPEC": "0"},
                                 {"ABNN_LEAN": "0"}, {"ABNN_GATE": "1024x16f32"}],
                         ids=["two-kernel", "spec-everywhere", "spec-off", "full-instance", "gate-1024x16"])
@pytest.mark.parametrize("over", [{}, dict(max_spikes=1), dict(max_spikes=200_000), dict(events=777_777),
                                  dict(max_spikes=5_000, base_scale=4.0)],
                         ids=["default", "budget1", "budget-huge", "partial", "dense-candidates"])
def test_pass_variants(gpu, monkeypatch, env, over):
    """The single-GPU pass's variants against the oracle every pass: the
    two-kernel pass (k_gate + k_apply, also the sharded and random-mode path),
    and the fused pass with its speculative weight stores everywhere (every
    workgroup past the budget's end restores its weights) or nowhere, with
    the full (not the lean) kernel instance, and with the
    1024x16 gate shape (the default is 1024x8).
    dense-candidates: the input->output records' ranges hold more spike
    candidates than a range lists (kCandCap), so the fused walk's list path,
    its fallback (every survivor) and a budget cut inside a range all run."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    over = dict(over)
    events = over.pop("events", 1_000_000)
    g, o = _pair(99_488, 1_000_000, events, seed=3, **over)
    for k in range(12):
        if k == 8:
            g.set_reward(0.5)
            o.set_reward(0.5)
        g.encode_traversal(1)
        o.pass_threaded(nthreads=16)
        _assert_same(g, o, f"{env} {over} pass {k}")
    assert g.stats() == o.stats()


def test_fused_and_shard_passes_interleaved(gpu):
    """One handle driven by fused passes (abnn_traverse) and world-1 shard
    passes (k_gate + k_apply) in turn: the bitmap buffers, the partition and
    the spike lists hand over between the two paths."""
    import torch

    g, o = _pair(99_488, 1_000_000, 1_000_000, seed=6)
    gs = GpuShards([g])
    for k in range(16):
        if k % 3 == 2 or k in (7, 8):
            gs.pass_()
        else:
            g.encode_traversal(1)
        torch.cuda.synchronize()
        o.pass_threaded(nthreads=16)
        _assert_same(g, o, f"pass {k}")
    assert g.stats() == o.stats()


def test_empty_and_tiny(gpu):
    import abnn_amd

    b = abnn_amd.Brain(256, 256, 10, 0, 1000)
    b.encode_traversal(3)
    assert b.scalars()["clock"] == 0  # brain.metal:61: no thread, no tick
    g, o = _pair(10, 1, 1)
    g.encode_traversal(6)
    o.pass_serial(6)
    _assert_same(g, o)


def test_inject_inputs_and_read_outputs(gpu):
    g, o = _pair(488, 10_000, 100_000, stim=False, seed=9)
    v = (np.arange(256) % 3 == 0).astype(np.float32) * 0.5
    for k in range(12):
        g.inject_inputs(v, 1000.0)
        o.inject_inputs(v, 1000.0)
        g.encode_traversal(1)
        o.pass_serial()
        assert np.array_equal(g.read_outputs(), o.read_outputs())
    _assert_same(g, o)
    g.set_timestamps([300, 301], 5)
    o.set_timestamps([300, 301], 5)
    assert np.array_equal(g.last_fired(), o.last_fired)


def _virtual_shard_run(world, n_syn, events, passes, n_hidden=30_000, seed=4):
    """`world` shard handles on one GPU driven phase by phase (what RCCL does across GPUs)."""
    import torch

    import abnn_amd
    from abnn_amd.shard import global_events, shard_ranges

    ge = global_events(n_syn, events, world)
    shards = []
    for lo, hi in shard_ranges(n_syn, world):
        b = abnn_amd.Brain(256, 256, n_hidden, hi - lo, events, syn_offset=lo, global_events=ge)
        b.build_random_graph(seed)
        b.set_auto_stimulus(0, 256)
        shards.append(b)
    gs = GpuShards(shards)
    for k in range(passes):
        if k == 6:
            for b in shards:
                b.set_reward(0.125)
        gs.pass_()
    torch.cuda.synchronize()
    return shards


@pytest.mark.parametrize("fused", ["1", "0"], ids=["fused-shard-pass", "two-kernel-shard-pass"])
@pytest.mark.parametrize("world", [2, 3])
def test_virtual_shards_equal_unsharded_gpu(gpu, monkeypatch, world, fused):
    """A sharded pass is k_gate (shard mode) + all-gather + k_shard_walk on the
    fused path, four kernels + all-gather on the two-kernel one: both equal
    the unsharded fused pass bit for bit."""
    monkeypatch.setenv("ABNN_FUSED", fused)
    n_syn, passes = 2_000_000, 10
    shards = _virtual_shard_run(world, n_syn, n_syn, passes)
    g, o = _pair(30_000, n_syn, n_syn, seed=4)
    for k in range(passes):
        if k == 6:
            g.set_reward(0.125)
        g.encode_traversal(1)
    syn = np.concatenate([b.download_synapses() for b in shards])
    assert np.array_equal(syn.view(np.uint32), g.download_synapses().view(np.uint32))
    for b in shards:
        assert np.array_equal(b.last_fired(), g.last_fired())
        assert b.scalars() == g.scalars()


def _flat_sections(path, n_nrn):
    raw = open(path, "rb").read()
    n = int(np.frombuffer(raw[:4], np.uint32)[0])
    pairs = np.frombuffer(raw[16:16 + 8 * n], np.uint32)
    w = np.frombuffer(raw[16 + 8 * n:16 + 12 * n], np.uint32)
    ts = raw[16 + 12 * n:]
    assert len(ts) == 16 * n_nrn
    return pairs, w, ts


@pytest.mark.parametrize("fused", ["1", "0"], ids=["fused-shard-pass", "two-kernel-shard-pass"])
@pytest.mark.parametrize("world", [2, 3])
def test_virtual_shards_visits_merge(gpu, monkeypatch, tmp_path, world, fused):
    """track_visits on shards: the lastVisited merge (abnn_shard_visits_delta /
    _merge after every renormalisation and before the read) equals the
    unsharded brain bit for bit, across two renormalisations and a host write
    ahead of the clock whose value pass 7's visits write again; so do the
    shards' flat saves (abnn_save_flat: records, lastFired, lastVisited)."""
    import torch

    import abnn_amd
    from abnn_amd.shard import global_events, shard_ranges
    from shard_helpers import merge_visits_local

    monkeypatch.setenv("ABNN_FUSED", fused)
    n_syn, passes, nh = 2_000_000, 9, 30_000
    kw = dict(track_visits=1, renorm_thresh=2)  # clock 0 1 2 3 | 0 1 2 3 | 0
    ge = global_events(n_syn, n_syn, world)
    shards = []
    for lo, hi in shard_ranges(n_syn, world):
        b = abnn_amd.Brain(256, 256, nh, hi - lo, n_syn, syn_offset=lo, global_events=ge, **kw)
        b.build_random_graph(4)
        b.set_auto_stimulus(0, 256)
        shards.append(b)
    g, o = _pair(nh, n_syn, n_syn, seed=4, **kw)
    gs = GpuShards(shards)
    for k in range(passes):
        if k == 4:
            for x in [g, o, *shards]:
                clk = x.scalars()["clock"]
                x.set_last_visited(np.full(8400, clk + 3, np.uint64), 600)
        g.encode_traversal(1)
        o.pass_serial()
        before = shards[0].renormalisations()
        gs.pass_()
        if shards[0].renormalisations() != before:
            merge_visits_local(shards)
    torch.cuda.synchronize()
    merge_visits_local(shards)
    assert g.renormalisations() == o.renormalisations() == shards[0].renormalisations() == 2
    assert np.array_equal(g.last_visited(), o.last_visited)
    _assert_same(g, o, "unsharded")
    g.save_flat(tmp_path / "whole.flat")
    wp, ww, wts = _flat_sections(tmp_path / "whole.flat", g.n_neuron())
    for r, ((lo, hi), b) in enumerate(zip(shard_ranges(n_syn, world), shards)):
        assert np.array_equal(b.last_visited(), g.last_visited()), f"rank {r} lastVisited"
        b.save_flat(tmp_path / f"shard{r}.flat")
        sp, sw, sts = _flat_sections(tmp_path / f"shard{r}.flat", b.n_neuron())
        assert np.array_equal(sp, wp[2 * lo:2 * hi]) and np.array_equal(sw, ww[lo:hi]), f"rank {r} records"
        assert sts == wts, f"rank {r} lastFired / lastVisited bytes"


def test_virtual_shards_partial_sweep_vs_oracle_shards(gpu):
    # events < shard size: each shard sweeps only its first `events` (config 4 shape)
    from abnn_amd.shard import global_events, shard_ranges
    from oracle import oracle as O

    world, n_syn, events, passes = 4, 4_000_000, 600_000, 9
    shards = _virtual_shard_run(world, n_syn, events, passes)
    ge = global_events(n_syn, events, world)
    obs = []
    for lo, hi in shard_ranges(n_syn, world):
        ob = O.OracleBrain(256, 256, 30_000, hi - lo, events, syn_offset=lo, global_events=ge)
        ob.build_random_graph(4, nthreads=16)
        ob.set_auto_stimulus(0, 256)
        obs.append(ob)
    for k in range(passes):
        if k == 6:
            for ob in obs:
                ob.set_reward(0.125)
        oracle_shard_pass(obs)
    for b, ob in zip(shards, obs):
        _assert_same(b, ob, "shard")


def test_save_load_roundtrips(gpu, tmp_path):
    import abnn_amd

    g, o = _pair(488, 10_000, 100_000)
    g.encode_traversal(9)
    p = tmp_path / "model.bnn"
    g.save(p)
    raw = p.read_bytes()
    assert len(raw) == 8 + 16 * 10_000
    assert np.frombuffer(raw[:8], dtype=np.uint32).tolist() == [10_000, 1000]  # brain.cpp:163-164
    h = abnn_amd.Brain(256, 256, 488, 10_000, 100_000)
    h.load(p)
    assert np.array_equal(h.download_synapses().view(np.uint32), g.download_synapses().view(np.uint32))
    bad = abnn_amd.Brain(256, 256, 489, 10_000, 100_000)
    with pytest.raises(abnn_amd.AbnnError) as e:
        bad.load(p)
    assert e.value.status == 4  # ABNN_ERR_SIZE_MISMATCH (brain.cpp:174 threw a pointer)
    f = tmp_path / "full.flat"
    g.save_flat(f)
    assert os.path.getsize(f) == 16 + 10_000 * 12 + 1000 * 16
    h2 = abnn_amd.Brain(256, 256, 488, 10_000, 100_000)
    h2.load_flat(f)
    assert np.array_equal(h2.download_synapses().view(np.uint32), g.download_synapses().view(np.uint32))
    assert np.array_equal(h2.last_fired(), g.last_fired())


def test_timing_and_stats_api(gpu):
    g, _ = _pair(99_488, 1_000_000, 1_000_000)
    g.enable_timing(True)
    g.encode_traversal(5)
    ms, n = g.kernel_time()
    assert n == 5 and ms > 0
    st = g.stats()
    assert st["passes"] == 5 and st["events"] == 5 * 1_000_000


@pytest.mark.slow
def test_config3_full_size_parity(gpu):
    """BASELINE configs[2] on one GPU: 5,000,512 neurons, 1B synapses (16 GB), 150M events.

    The sweep touches only the first E = 150,000,128 records, so the CPU oracle
    holds just those; everything else is checked by the additive checksum."""
    import abnn_amd
    from oracle import oracle as O

    n_hidden, n_syn, events = 5_000_000, 1_000_000_000, 150_000_000
    g = abnn_amd.Brain(256, 256, n_hidden, n_syn, events)
    g.build_random_graph(1)
    E = g.visited_events()
    assert E == 150_000_128
    ck_cpu = 0
    step = 50_000_000
    for first in range(0, n_syn, step):
        part = O.gen_synapses(first, min(step, n_syn - first), 256, 256, 5_000_512, 1, nthreads=16)
        ck_cpu = (ck_cpu + O.checksum(part, first)) % (1 << 64)
    del part
    assert g.checksum() == ck_cpu
    o = O.OracleBrain(256, 256, n_hidden, E, events)
    o.build_random_graph(1, nthreads=16)
    g.set_auto_stimulus(0, 256)
    o.set_auto_stimulus(0, 256)
    g.encode_traversal(8)
    o.pass_threaded(8, nthreads=16)
    head = g.download_synapses(0, E)
    assert np.array_equal(head.view(np.uint32), o.syn.view(np.uint32))
    assert np.array_equal(g.last_fired(), o.last_fired)
    assert g.scalars()["clock"] == o.clock
    st_g, st_o = g.stats(), o.stats()
    assert st_g == st_o


def _bitmap(g):
    import ctypes as C
    nw = 2 * ((g.n_neuron() + 63) // 64)
    out = np.zeros(nw, dtype=np.uint32)
    inc = C.c_int(0)
    f = g._lib.abnn_debug_bitmap
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_int)]
    f.restype = C.c_int
    assert f(g._h, out.ctypes.data, nw, C.byref(inc)) == 0
    return out, bool(inc.value)


def _expected_bitmap(last_fired_at_start, now, n_words, window=5):
    bits = ((np.uint64(now) - last_fired_at_start.astype(np.uint64)) <= np.uint64(window)).astype(np.uint8)
    bits = np.concatenate([bits, np.zeros(n_words * 32 - bits.size, np.uint8)])
    return np.packbits(bits.reshape(-1, 32)[:, ::-1], axis=1).view(">u4").ravel().astype(np.uint32)


def test_recent_bitmap_update_with_host_writes(gpu):
    """The steady-state bitmap (built by k_apply from the last passes' spike
    lists) against the bitmap recomputed from lastFired every pass, and the
    whole state against the oracle, across the host writes that force k_bitmap
    rebuilds: set_timestamps, set_last_fired (recent and future values), a
    clock jump."""
    g, o = _pair(99_488, 1_000_000, 1_000_000)
    modes = []
    for k in range(34):
        now = g.scalars()["clock"]
        lf0 = g.last_fired()  # lastFired at pass start, host writes included
        if k == 12:
            g.set_timestamps([300, 5000, 77_000], now)
            o.set_timestamps([300, 5000, 77_000], now)
            lf0[[300, 5000, 77_000]] = now
        if k == 18:
            v = np.full(1000, now - 2, np.uint64)
            v[::7] = now + 3  # not recent until the clock gets there
            g.set_last_fired(v, 40_000)
            o.last_fired[40_000:41_000] = v
            lf0[40_000:41_000] = v
        if k == 24:
            sc = g.scalars()
            g.set_scalars(sc["clock"] + 100, sc["reward"], sc["rbar"], sc["pass_index"])
            so = o.scalars()
            o.set_scalars(so["clock"] + 100, so["reward"], so["rbar"], so["pass_index"])
            now += 100
        lf0[:256] = now  # the stimulus is stamped at pass start
        g.encode_traversal(1)
        o.pass_threaded(nthreads=16)
        bm, inc_next = _bitmap(g)
        modes.append(inc_next)
        assert np.array_equal(bm, _expected_bitmap(lf0, now, bm.size)), f"bitmap, pass {k}"
        _assert_same(g, o, f"pass {k}")
    assert all(modes[5:12]) and all(modes[28:]), modes  # built by k_apply before and after the writes
    assert not any(modes[12:17]) and not any(modes[18:28]), modes
