"""CPU tests of the oracle: known answers, restatement cross-check, threaded and
sharded phases vs the serial C1 loop.  (Parity against the reference itself is
UNPINNED -- DESIGN.md §3.)"""
import numpy as np
import pytest

from oracle import oracle as O
from py_reference import MetalEmu, rand01 as py_rand01
from shard_helpers import oracle_shard_pass

PARAMS = dict(base_scale=0.8, refractory=2, window_pre=5, clock_inc=1, target_rate_hz=1000.0,
              eta_home=1e-6, eta_reward=1e-3, alpha_rbar=0.001, a_ltp=0.04, a_ltd=0.02,
              w_min=0.001, w_max=1.0, max_spikes=2560, renorm_thresh=4_000_000)


def test_rand01_known_answers():
    # brain.metal:15-19 by hand: s=1 -> 1^(1<<13)=8193 -> ^>>17 = 8193 -> ^(8193<<5)=270369
    assert O.rand01(0) == 0.0
    assert O.rand01(1) == np.float32(270369 / 16777216.0)
    for s in [2, 3, 12345, 0xFFFFFFFF, 0x80000000, 0xDEADBEEF]:
        assert O.rand01(s) == float(py_rand01(s))


def test_default_params_match_reference_constants():
    p = O.default_params()
    assert np.float32(p.base_scale) == np.float32(0.8)
    assert (p.refractory, p.window_pre, p.clock_inc, p.max_spikes) == (2, 5, 1, 2560)
    assert np.float32(p.a_ltp) == np.float32(0.04) and np.float32(p.a_ltd) == np.float32(0.02)
    assert np.float32(p.w_min) == np.float32(0.001) and p.w_max == 1.0
    assert p.renorm_thresh == 4_000_000 and (p.tau_vis, p.tau_pre) == (50_000, 50_000)


def test_generator_recipe():
    n_in, n_out, n_nrn = 256, 256, 100_000
    s = O.gen_synapses(0, 200_000, n_in, n_out, n_nrn, seed=1, nthreads=4)
    dense = s[: n_in * n_out]
    idx = np.arange(n_in * n_out)
    assert np.array_equal(dense["src"], idx // n_out)
    assert np.array_equal(dense["dst"], n_in + idx % n_out)
    assert dense["w"].min() >= np.float32(0.4) and dense["w"].max() < np.float32(0.8)
    hid = s[n_in * n_out:]
    assert hid["src"].min() >= 512 and hid["src"].max() < n_nrn
    assert hid["dst"].min() >= 512 and hid["dst"].max() < n_nrn
    assert hid["w"].min() >= np.float32(0.1) and hid["w"].max() < np.float32(0.2)
    assert np.all(s["pad"] == 0)
    # counter-based: any slice is reproducible independently, any thread count
    part = O.gen_synapses(123_457, 1000, n_in, n_out, n_nrn, seed=1, nthreads=1)
    assert np.array_equal(part.view(np.uint32), s[123_457:124_457].view(np.uint32))
    other = O.gen_synapses(0, 1000, n_in, n_out, n_nrn, seed=2)
    assert not np.array_equal(other.view(np.uint32), s[:1000].view(np.uint32))


def test_checksum_is_position_sensitive():
    s = O.gen_synapses(0, 5000, 256, 256, 1000, seed=1)
    c = O.checksum(s)
    s2 = s.copy()
    s2[[10, 11]] = s2[[11, 10]]
    assert O.checksum(s2) != c
    s3 = s.copy()
    s3["w"][4999] = np.nextafter(s3["w"][4999], np.float32(1))
    assert O.checksum(s3) != c
    assert O.checksum(s[100:], first_global=100) + O.checksum(s[:100]) == c


def _emu_from(ob: O.OracleBrain, events):
    p = dict(PARAMS)
    for k in p:
        p[k] = getattr(ob.p, k)
    p["track_visits"] = ob.p.track_visits
    p["mode"], p["seed"] = ob.p.mode, ob.p.seed
    e = MetalEmu(ob.syn["src"], ob.syn["dst"], ob.syn["w"], ob.n_neuron(), events, p)
    return e


def _compare(ob, emu):
    assert ob.clock == emu.clock
    assert np.array_equal(ob.last_fired, np.array(emu.lastF, dtype=np.uint64))
    w = np.array(emu.w, dtype=np.float32)
    assert np.array_equal(ob.syn["w"].view(np.uint32), w.view(np.uint32))
    assert np.float32(ob.s.rbar) == emu.rbar


@pytest.mark.parametrize("case", ["c1", "hidden", "reward", "renorm", "visits"])
def test_serial_oracle_matches_python_restatement(case):
    n_hidden, n_syn, events, passes = 488, 10_000, 100_000, 10
    over = {}
    if case == "hidden":
        n_hidden, n_syn, events, passes = 3000, 90_000, 20_000, 9
    if case == "renorm":
        over["renorm_thresh"] = 4
        passes = 12
    if case == "visits":
        over["track_visits"] = 1
    ob = O.OracleBrain(256, 256, n_hidden, n_syn, events, **over)
    ob.build_random_graph(seed=7)
    ob.set_auto_stimulus(0, 256)
    emu = _emu_from(ob, events)
    emu.stim = (0, 256)
    for k in range(passes):
        if case == "reward" and k == 4:
            ob.set_reward(0.75)
            emu.reward = np.float32(0.75)
        ob.pass_serial()
        emu.one_pass()
        _compare(ob, emu)
    if case == "visits":
        assert np.array_equal(ob.last_visited, np.array(emu.lastV, dtype=np.uint64))
    if case == "renorm":
        assert ob.clock < 10  # renormalised at least once


def _run(kind, nthreads=1, world=1, passes=8, **kw):
    n_hidden = kw.pop("n_hidden", 20_000)
    n_syn = kw.pop("n_syn", 300_000)
    events = kw.pop("events", 250_000)
    ob = O.OracleBrain(256, 256, n_hidden, n_syn, events, **kw)
    ob.build_random_graph(seed=3)
    ob.set_auto_stimulus(0, 256)
    for k in range(passes):
        if k == 5:
            ob.set_reward(-0.5)
        if kind == "serial":
            ob.pass_serial()
        else:
            ob.pass_threaded(nthreads=nthreads)
    return ob


@pytest.mark.parametrize("nthreads", [1, 2, 3, 8, 17])
def test_threaded_equals_serial(nthreads):
    a = _run("serial")
    b = _run("threaded", nthreads=nthreads)
    assert a.clock == b.clock
    assert np.array_equal(a.syn.view(np.uint32), b.syn.view(np.uint32))
    assert np.array_equal(a.last_fired, b.last_fired)
    assert np.float32(a.s.rbar) == np.float32(b.s.rbar)
    sa, sb = a.stats(), b.stats()
    assert sa == sb


def test_threaded_equals_serial_small_budget_and_edges():
    for kw in [dict(max_spikes=1), dict(max_spikes=0), dict(max_spikes=1_000_000),
               dict(events=1), dict(events=300_000 + 1000), dict(refractory=0, window_pre=0)]:
        a = _run("serial", passes=7, **dict(kw))
        b = _run("threaded", nthreads=5, passes=7, **dict(kw))
        assert np.array_equal(a.syn.view(np.uint32), b.syn.view(np.uint32)), kw
        assert np.array_equal(a.last_fired, b.last_fired), kw
        assert a.clock == b.clock, kw


def test_empty_graph_never_ticks():
    ob = O.OracleBrain(256, 256, 10, 0, 1000)
    ob.pass_serial(3)
    assert ob.clock == 0  # brain.metal:61 returns before any tick
    ob2 = O.OracleBrain(256, 256, 10, 100, 0)
    ob2.pass_serial(2)
    assert ob2.clock == 0  # empty grid


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_shard_phases_equal_serial_full_sweep(world):
    # events >= shard size: every shard sweeps its whole range -> global order = unsharded full sweep
    n_syn = 300_000
    shards = _sharded_full(world)
    ref = _run("serial", passes=8, n_hidden=20_000, n_syn=n_syn, events=n_syn)
    syn = np.concatenate([s.syn for s in shards])
    assert np.array_equal(syn.view(np.uint32), ref.syn.view(np.uint32))
    for s in shards:
        assert np.array_equal(s.last_fired, ref.last_fired)
        assert s.clock == ref.clock
        assert np.float32(s.s.rbar) == np.float32(ref.s.rbar)


def _sharded_full(world, passes=8):
    from abnn_amd.shard import shard_ranges, global_events

    n_hidden, n_syn, events = 20_000, 300_000, 300_000
    ge = global_events(n_syn, events, world)
    shards = []
    for lo, hi in shard_ranges(n_syn, world):
        ob = O.OracleBrain(256, 256, n_hidden, hi - lo, events, syn_offset=lo, global_events=ge)
        ob.build_random_graph(seed=3)
        ob.set_auto_stimulus(0, 256)
        shards.append(ob)
    for k in range(passes):
        if k == 5:
            for ob in shards:
                ob.set_reward(-0.5)
        oracle_shard_pass(shards)
    return shards


def test_inject_and_read_outputs():
    ob = O.OracleBrain(256, 256, 488, 10_000, 100_000)
    ob.build_random_graph(seed=1)
    v = np.zeros(256, dtype=np.float32)
    v[::3] = 0.5
    ob.s.clock = 7
    ob.inject_inputs(v, 1000.0)
    fired = np.nonzero(ob.last_fired[:256] == 7)[0]
    assert np.array_equal(fired, np.arange(0, 256, 3))  # pTick ~ 1e15: every v>0 fires
    ob.last_fired[256 + 5] = 7
    ob.last_fired[256 + 6] = 6
    ob.s.clock = 8
    out = ob.read_outputs()
    assert out[5] and not out[6] and out.sum() == 1


# ---- random-edge mode (README §4; build-defined contract in include/abnn/abnn.h) ----

def test_philox_known_answers():
    """The published Philox4x32-10 known-answer vectors (Random123 kat_vectors)."""
    from py_reference import philox4x32_10 as py_philox

    kat = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
           ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
           ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
            (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]
    for ctr, key, want in kat:
        assert tuple(O.philox4x32_10(ctr, key)) == want
        assert tuple(py_philox(ctr, key)) == want


def test_pick_in_range_and_uniform():
    from py_reference import pick as py_pick

    n = 1000
    picks = np.array([O.pick(7, 0, 3, t, n) for t in range(20_000)])
    assert picks.min() >= 0 and picks.max() < n
    counts = np.bincount(picks, minlength=n)
    assert counts.min() > 0 and abs(counts.mean() - 20.0) < 1e-9 and counts.std() < 7.0
    for t in (0, 1, 123456, 2**32 + 5):
        for stream, pidx, nn in ((0, 0, 10), (99, 2**33, 4_000_000_000), (5, 1, 1)):
            assert O.pick(11, stream, pidx, t, nn) == py_pick(11, stream, pidx, t, nn)


def _random_brain(n_hidden=488, n_syn=2_000, events=12_000, **kw):
    ob = O.OracleBrain(256, 256, n_hidden, n_syn, events, mode=1, seed=9, **kw)
    ob.build_random_graph(seed=5)
    ob.set_auto_stimulus(0, 256)
    return ob


@pytest.mark.parametrize("case", ["dense", "hidden", "visits"])
def test_random_mode_oracle_matches_python_restatement(case):
    # n_syn << events: ~6 visits per synapse per pass, so colliding updates are common
    kw = {"n_hidden": 3000, "n_syn": 30_000, "events": 9_000} if case == "hidden" else {}
    if case == "visits":
        kw["track_visits"] = 1
    ob = _random_brain(**kw)
    emu = _emu_from(ob, ob.s.dims.events_per_pass)
    emu.p["mode"], emu.p["seed"] = 1, 9
    emu.stim = (0, 256)
    for k in range(8):
        if k == 4:
            ob.set_reward(0.6)
            emu.reward = np.float32(0.6)
        ob.pass_serial()
        emu.one_pass()
        _compare(ob, emu)
    assert ob.scalars()["pass_index"] == 8 and ob.stats()["events"] == 8 * ob.s.dims.events_per_pass
    if case == "visits":
        assert np.array_equal(ob.last_visited, np.array(emu.lastV, dtype=np.uint64))


def test_random_mode_collisions_happen():
    ob = _random_brain()
    E, n = int(ob.s.dims.events_per_pass), int(ob.s.dims.n_syn)
    picks = [O.pick(9, 0, 0, t, n) for t in range(E)]
    assert len(set(picks)) < E  # the collision rule is exercised


@pytest.mark.parametrize("nthreads", [1, 3, 8])
def test_random_mode_threaded_equals_serial(nthreads):
    a, b = _random_brain(), _random_brain()
    for _ in range(7):
        a.pass_serial()
        b.pass_threaded(nthreads=nthreads)
    assert np.array_equal(a.syn.view(np.uint32), b.syn.view(np.uint32))
    assert np.array_equal(a.last_fired, b.last_fired)
    assert a.scalars() == b.scalars() and a.stats() == b.stats()


def test_random_mode_shard_phases_world1_equal_serial():
    a, b = _random_brain(), _random_brain()
    for _ in range(6):
        a.pass_serial()
        oracle_shard_pass([b])
    assert np.array_equal(a.syn.view(np.uint32), b.syn.view(np.uint32))
    assert np.array_equal(a.last_fired, b.last_fired)
    assert a.scalars() == b.scalars()


# ---- structural plasticity (README §5; build-defined contract in include/abnn/abnn.h) ----

SP = dict(w_prune=0.105, p_new=0.35, w_init=0.5, compact_every=2)


def _sp_brain(mode=0, cap_extra=20_000, n_hidden=3000, n_syn=120_000, events=120_000, **over):
    kw = dict(SP)
    kw.update(over)
    ob = O.OracleBrain(256, 256, n_hidden, n_syn, events, mode=mode, seed=13,
                       syn_capacity=n_syn + cap_extra, **kw)
    ob.build_random_graph(seed=21)
    ob.set_auto_stimulus(0, 256)
    return ob


# sweep of the whole array (the tail shifts down), a sweep of its first third
# (the hole takes the array's last records), random picks
@pytest.mark.parametrize("mode,events", [(0, 120_000), (0, 90_000), (1, 30_000)])
def test_structural_plasticity_matches_python_restatement(mode, events):
    ob = _sp_brain(mode, events=events, track_visits=1)
    emu = _emu_from(ob, ob.s.dims.events_per_pass)
    emu.p.update(SP)
    emu.p["track_visits"] = 1
    emu.capacity = int(ob.s.dims.syn_capacity)
    emu.stim = (0, 256)
    n0 = ob.n_syn = None
    sizes = []
    for k in range(9):
        if k == 5:
            ob.set_reward(0.4)
            emu.reward = np.float32(0.4)
        ob.pass_serial()
        emu.one_pass()
        sizes.append(int(ob.s.dims.n_syn))
        assert int(ob.s.dims.n_syn) == len(emu.src), k
        assert np.array_equal(ob.syn["src"], np.array(emu.src, dtype=np.uint32)), k
        assert np.array_equal(ob.syn["dst"], np.array(emu.dst, dtype=np.uint32)), k
        _compare(ob, emu)
        assert np.array_equal(ob.last_visited, np.array(emu.lastV, dtype=np.uint64)), k
    st = ob.stats()
    assert st["pruned"] == emu.pruned > 0 and st["grown"] == emu.n_grown > 0
    assert len(set(sizes)) > 1  # the graph changed size


@pytest.mark.parametrize("tombs,expect", [
    # D = 2, m = 18: the holes 2 and 4 take the tail's 18 and 19
    ([2, 4], [0, 1, 18, 3, 19] + list(range(5, 18))),
    # the first record: its hole takes the last one
    ([0], [19] + list(range(1, 19))),
    # D = 3, m = 17, tombstones in the tail too: the hole 15 takes the tail's
    # only live record, 19; 17 and 18 lie in the tail and just go
    ([15, 17, 18], list(range(15)) + [19, 16]),
    # the last record: nothing below m to fill
    ([19], list(range(19))),
    # every record
    (list(range(20)), []),
    # D = 4, m = 16: holes 0, 7 take 16, 19 (17 is in the tail, 18 too)
    ([0, 7, 17, 18], [16] + list(range(1, 7)) + [19] + list(range(8, 16))),
])
def test_structural_update_removal_contract(tombs, expect):
    """The removal of abnn.h's structural update on a hand-made array (no
    pass work: 0 events, an update after every pass): with D tombstones the
    array ends at m = n - D, and the tombstones below m take, in order, the
    live records of the tail [m, n) in order."""
    ob = O.OracleBrain(256, 256, 100, 20, 0, compact_every=1, w_prune=0.1, syn_capacity=20)
    syn = np.zeros(20, dtype=O.SYN_DTYPE)
    syn["src"] = 256 + np.arange(20)
    syn["dst"] = np.arange(20)  # record identity
    syn["w"] = 0.5
    syn["src"][tombs] = 0xFFFFFFFF
    syn["dst"][tombs] = 0xFFFFFFFF
    ob.set_synapses(syn)
    ob.pass_serial()
    assert int(ob.s.dims.n_syn) == len(expect)
    assert ob.syn["dst"].tolist() == expect


def test_structural_update_is_not_the_stable_compaction():
    """Deliberate change from round 4 (structural update): the
    stable compaction of the whole array is a non-goal.  Where the two orders
    differ, the records a sweep's visited window [0, events) holds after the
    update differ too: here the window of 5 takes records 18, 19 (the holes'
    fill), where the stable order would have given 5, 6."""
    ob = O.OracleBrain(256, 256, 100, 20, 5, compact_every=1, w_prune=0.1, syn_capacity=20)
    syn = np.zeros(20, dtype=O.SYN_DTYPE)
    syn["src"] = 256 + np.arange(20)
    syn["dst"] = np.arange(20)
    syn["w"] = 0.5
    syn["src"][[2, 4]] = 0xFFFFFFFF
    syn["dst"][[2, 4]] = 0xFFFFFFFF
    ob.set_synapses(syn)
    ob.pass_serial()
    got = ob.syn["dst"].tolist()
    stable = [i for i in range(20) if i not in (2, 4)]
    assert sorted(got) == stable and got != stable
    assert got[:5] == [0, 1, 18, 3, 19] and stable[:5] == [0, 1, 3, 5, 6]


def test_structural_update_semantics():
    ob = _sp_brain(0)
    n_nrn = ob.n_neuron()
    for _ in range(8):
        ob.pass_serial()
    s = ob.syn
    live = s["src"] != 0xFFFFFFFF
    # odd number of passes since the last update would leave tombstones; after an
    # even pass count (compact_every = 2) every tombstone has been compacted away
    assert live.all()
    grown = s[s["w"] == np.float32(0.5)]
    assert grown.shape[0] > 0 and (grown["dst"] >= 256).all() and (grown["dst"] < n_nrn).all()
    assert ob.stats()["grown"] >= grown.shape[0] - 10  # (a few original weights may be 0.5 exactly)
    assert int(ob.s.dims.n_syn) <= int(ob.s.dims.syn_capacity)


def test_structural_capacity_caps_growth():
    ob = _sp_brain(0, cap_extra=0, w_prune=0.0)  # nothing is removed, nothing can be added
    n0 = int(ob.s.dims.n_syn)
    for _ in range(6):
        ob.pass_serial()
    assert int(ob.s.dims.n_syn) == n0 and ob.stats()["grown"] == 0 and ob.stats()["pruned"] == 0


@pytest.mark.parametrize("mode,nthreads", [(0, 1), (0, 5), (1, 4)])
def test_structural_threaded_equals_serial(mode, nthreads):
    a, b = _sp_brain(mode), _sp_brain(mode)
    for _ in range(7):
        a.pass_serial()
        b.pass_threaded(nthreads=nthreads)
    assert int(a.s.dims.n_syn) == int(b.s.dims.n_syn)
    assert np.array_equal(a.syn.view(np.uint32), b.syn.view(np.uint32))
    assert np.array_equal(a.last_fired, b.last_fired)
    assert a.scalars() == b.scalars() and a.stats() == b.stats()


@pytest.mark.parametrize("mode", [0, 1])
def test_structural_shard_world1_equals_serial(mode):
    a, b = _sp_brain(mode), _sp_brain(mode)
    for _ in range(6):
        a.pass_serial()
        oracle_shard_pass([b])
    assert np.array_equal(a.syn.view(np.uint32), b.syn.view(np.uint32))
    assert a.stats() == b.stats()


def test_stamp_ahead_of_clock_ages_in_u32():
    """lastF/clock are `uint` in the reference (brain.metal:43,45): a dst stamp
    ahead of the clock (a host write of now + 3) is 2^32 - 3 ticks old, not
    2^64 - 3 (brain.metal:80,116).  isi = float(2^32 - 3) = 2^32, so the
    homeostatic term 1000 - 1e6/isi is 999.99976f (not 1000.0f)."""
    f = np.float32
    isi = f(2**32 - 3)
    assert isi == f(2**32)
    est = f(f(1e6) / isi)
    assert f(f(1000.0) - est) == f(999.99976)
    assert f(f(1000.0) - f(f(1e6) / f(2.0**64))) == f(1000.0)  # what u64 ages would give

    now = 100
    ob = O.OracleBrain(1, 1, 1, 1, 1)
    ob.set_synapses(np.array([(0, 1, 0.3, 0.0)], dtype=O.SYN_DTYPE))
    ob.set_scalars(now, 0.0, 0.0, 0)
    ob.last_fired[:] = [now, now + 3, 0]        # pre-spike recent; dst stamped ahead of the clock
    w = f(0.3)
    cand = f(f(w * w) * f(0.8)) > f(O.rand01(0 ^ now))
    ob.pass_serial(1)
    st = ob.stats()
    assert (st["pre_gated"], st["post_gated"], st["updated"]) == (1, 1, 1)  # 2^32-3 > REFRACTORY
    dW = f(f(0.04) * f(f(1.0) - w)) if cand else f(f(-0.02) * w)
    dW = f(dW + f(f(f(1e-3) * f(0.0)) * f(1.0 if cand else 0.0)))
    dW = f(dW + f(f(f(1e-6) * f(999.99976)) * w))
    expect = min(max(f(w + dW), f(0.001)), f(1.0))
    assert ob.syn["w"][0].view(np.uint32) == np.float32(expect).view(np.uint32)
    # the emulator (per-thread Metal semantics) agrees
    emu = _emu_from(O.OracleBrain(1, 1, 1, 1, 1), 1)
    emu.src, emu.dst, emu.w = [0], [1], [f(0.3)]
    emu.clock = now
    emu.lastF = [now, now + 3, 0]
    emu.one_pass()
    assert np.float32(emu.w[0]).view(np.uint32) == np.float32(expect).view(np.uint32)


def test_read_outputs_and_renorm_use_u32_clock():
    """read_outputs (brain.cpp:149-154) and the renormalisation test
    (brain.cpp:127-128) compare u32 values."""
    ob = O.OracleBrain(1, 2, 0, 1, 1)
    ob.set_scalars((1 << 32) + 5, 0.0, 0.0, 0)
    ob.last_fired[:] = [0, 4, (1 << 33) + 4]  # both outputs stamped at (u32) now - 1
    assert list(ob.read_outputs()) == [True, True]
