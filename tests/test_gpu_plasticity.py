"""GPU parity of structural plasticity (README §5; contract in include/abnn/abnn.h):
pruning to tombstones in k_apply, synaptogenesis into per-pass budget slots,
and the structural update (the tombstones' span closed up, its hole filled
from the array's end, then the ordered append; abnn.h) -- HIP path vs
the CPU oracle, bit-exact, pass by pass, record count included.  No reference
code exists for this; the oracle is cross-checked against an independent
Python restatement in tests/test_oracle.py."""
import numpy as np
import pytest

from shard_helpers import GpuShards, oracle_shard_pass

pytestmark = pytest.mark.gpu

SP = dict(w_prune=0.105, p_new=0.35, w_init=0.5, compact_every=2)


def _pair(mode=0, n_hidden=3000, n_syn=120_000, events=120_000, cap_extra=20_000, syn_offset=0,
          global_events=0, **over):
    import abnn_amd
    from oracle import oracle as O

    kw = dict(SP, mode=mode, seed=13)
    kw.update(over)
    cap = n_syn + cap_extra
    g = abnn_amd.Brain(256, 256, n_hidden, n_syn, events, syn_offset=syn_offset,
                       global_events=global_events, syn_capacity=cap, **kw)
    o = O.OracleBrain(256, 256, n_hidden, n_syn, events, syn_offset=syn_offset,
                      global_events=global_events, syn_capacity=cap, **kw)
    g.build_random_graph(21)
    o.build_random_graph(21, nthreads=16)
    g.set_auto_stimulus(0, 256)
    o.set_auto_stimulus(0, 256)
    return g, o


def _same(g, o, what=""):
    assert g.n_syn() == int(o.s.dims.n_syn), f"n_syn {what}"
    assert np.array_equal(g.download_synapses().view(np.uint32), o.syn.view(np.uint32)), f"synapses {what}"
    assert np.array_equal(g.last_fired(), o.last_fired), f"lastFired {what}"
    sg, so = g.scalars(), o.scalars()
    assert sg["clock"] == so["clock"] and sg["pass_index"] == so["pass_index"], what
    assert np.float32(sg["rbar"]) == np.float32(so["rbar"]), what


@pytest.mark.parametrize("mode", [0, 1])
def test_plasticity_every_pass(gpu, mode):
    g, o = _pair(mode, events=120_000 if mode == 0 else 60_000)
    sizes = set()
    for k in range(12):
        if k == 6:
            g.set_reward(0.4)
            o.set_reward(0.4)
        g.encode_traversal(1)
        o.pass_serial()
        _same(g, o, f"pass {k}")
        sizes.add(g.n_syn())
    st = g.stats()
    assert st == o.stats()
    assert st["pruned"] > 0 and st["grown"] > 0 and len(sizes) > 1
    assert g.visited_events() == (min(g.n_syn(), 120_064) if mode == 0 else 60_000)


@pytest.mark.parametrize("ce", [1, 3])
def test_plasticity_compact_schedule(gpu, ce):
    g, o = _pair(0, compact_every=ce)
    for k in range(7):
        g.encode_traversal(1)
        o.pass_threaded(nthreads=16)
        _same(g, o, f"pass {k}")
    assert g.stats() == o.stats()


def test_plasticity_large_with_visits(gpu):
    g, o = _pair(0, n_hidden=99_488, n_syn=1_000_000, events=1_000_000, cap_extra=100_000,
                 track_visits=1)
    for _ in range(8):
        g.encode_traversal(1)
        o.pass_threaded(nthreads=16)
    _same(g, o)
    assert np.array_equal(g.last_visited(), o.last_visited)
    assert g.stats() == o.stats()


@pytest.mark.parametrize("fmt", ["bnn", "flat", "upload"])
def test_pruned_brain_round_trips_before_its_structural_update(gpu, tmp_path, fmt):
    """A pruned brain holds tombstones {src = dst = 0xFFFFFFFF} until its next
    structural update; saving it there and loading the file into a fresh
    handle must work and the structural update of the loaded
    brain must compact exactly like the original's (its tombstone tally is
    recounted from the loaded records)."""
    import abnn_amd

    kw = dict(p_new=0.0, compact_every=8)
    g, o = _pair(0, **kw)
    for _ in range(6):  # passes 3-5 prune; no structural update yet (pass_index 6 % 8)
        g.encode_traversal(1)
        o.pass_serial()
    syn = g.download_synapses()
    tomb = (syn["src"] == 0xFFFFFFFF) & (syn["dst"] == 0xFFFFFFFF)
    assert tomb.any() and g.n_syn() == 120_000
    h = abnn_amd.Brain(256, 256, 3000, 120_000, 120_000, syn_capacity=140_000, **dict(SP, seed=13, **kw))
    if fmt == "bnn":
        g.save(tmp_path / "m.bnn")
        h.load(tmp_path / "m.bnn")
    elif fmt == "flat":
        g.save_flat(tmp_path / "m.flat")
        h.load_flat(tmp_path / "m.flat")
    else:
        h.upload_synapses(syn)
    if fmt != "flat":
        h.set_last_fired(g.last_fired())
    s = g.scalars()
    h.set_scalars(s["clock"], s["reward"], s["rbar"], s["pass_index"])
    h.set_auto_stimulus(0, 256)
    assert np.array_equal(h.download_synapses().view(np.uint32), syn.view(np.uint32))
    for k in range(4):  # through the structural update after pass_index 8
        h.encode_traversal(1)
        o.pass_serial()
        _same(h, o, f"{fmt} pass {k}")
    assert h.n_syn() < 120_000


def test_plasticity_virtual_shards_vs_oracle_shards(gpu):
    import torch

    from abnn_amd.shard import global_events, shard_ranges

    world, n_syn, events, passes = 2, 240_000, 240_000, 8
    ge = global_events(n_syn, events, world)
    pairs = [_pair(0, n_syn=hi - lo, events=events, syn_offset=lo, global_events=ge)
             for lo, hi in shard_ranges(n_syn, world)]
    gs = GpuShards([g for g, _ in pairs])
    for k in range(passes):
        gs.pass_()
        oracle_shard_pass([o for _, o in pairs])
    torch.cuda.synchronize()
    for g, o in pairs:
        _same(g, o, "shard")
        assert g.stats() == o.stats()


@pytest.mark.parametrize("pattern", ["spread", "dense_block", "tail_short", "almost_all"])
def test_structural_update_in_place_patterns(gpu, pattern):
    """The device-driven structural update (kernels.hip launch_structural_update:
    the holes' ranks, the tail's live prefix, the holes filled from the tail)
    on uploaded tombstone patterns the passes' pruning does not produce --
    tombstones everywhere incl. the first and last record (the tail holds
    tombstones: the tail-scan path), a dense run of 50k (12 whole blocks of
    holes) plus a spread (the tail is live: the direct path), a run at the
    end that reaches below m, and all but every 1000th record -- against the
    oracle's restatement of the contract (abnn.h), records and count after
    each update."""
    kw = dict(w_prune=1e-30, p_new=0.0, compact_every=1)  # the passes prune nothing; the update removes the uploads'
    g, o = _pair(0, **kw)
    syn = g.download_synapses()
    n = len(syn)
    idx = np.arange(n)
    dead = {"spread": (idx % 7 == 3) | (idx == 0) | (idx == n - 1),
            "dense_block": (idx >= 10_000) & (idx < 60_000) | (idx % 97 == 5),
            "tail_short": (idx >= 100_000) & (idx < 118_000),
            "almost_all": idx % 1000 != 17}[pattern]
    syn["src"][dead] = 0xFFFFFFFF
    syn["dst"][dead] = 0xFFFFFFFF
    g.upload_synapses(syn)
    o.set_synapses(syn)
    for k in range(2):
        g.encode_traversal(1)
        o.pass_serial()
        _same(g, o, f"{pattern} pass {k}")
    assert g.n_syn() <= n - int(dead.sum())


def _hip_copy_d2d(dst: int, src: int, nbytes: int) -> None:
    """hipMemcpy device -> device through the runtime torch loaded (test-only raw write)."""
    import ctypes as C
    import os

    import torch

    hip = C.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    assert hip.hipMemcpy(dst, src, nbytes, 3) == 0  # hipMemcpyDeviceToDevice
    assert hip.hipDeviceSynchronize() == 0


def test_failed_structural_update_refuses_passes(gpu, tmp_path):
    """A structural update that fails part-way leaves the records invalid (the
    holes' fill moves records in place), so the handle then refuses every
    pass (ABNN_ERR_INVALID) until they are reloaded.  The failure the fill
    detects: a tombstone tally that disagrees with the records (the last
    tallied block's tombstones revived behind the handle's back through the
    device layout).  (Round 5's second case, a compaction wait that gave up,
    has no counterpart: the round-6 fill waits on no other workgroup.)  After
    a reload the passes equal the oracle again."""
    from abnn_amd import _lib

    kw = dict(w_prune=1e-30, p_new=0.0, compact_every=1)
    g, o = _pair(0, **kw)
    syn = g.download_synapses()
    idx = np.arange(len(syn))
    dead = (idx >= 10_000) & (idx < 60_000)
    syn["src"][dead] = 0xFFFFFFFF
    syn["dst"][dead] = 0xFFFFFFFF
    g.upload_synapses(syn)
    o.set_synapses(syn)
    flat, sc = str(tmp_path / "before.flat"), g.scalars()
    g.save_flat(flat)

    def refused():
        with pytest.raises(_lib.AbnnError, match="failed structural update") as e:
            g.encode_traversal(1)
        assert e.value.status == 1  # ABNN_ERR_INVALID

    def reload():
        g.load_flat(flat)
        g.set_scalars(sc["clock"], sc["reward"], sc["rbar"], sc["pass_index"])

    # (2) records [57344, 60160) (the last tallied block's tombstones, whole
    # 256-record groups) revived with the codes and {dst, w} of records [0, 2816)
    lay = g.synapse_layout()["arrays"]
    a, m = 57344, 2816
    for name, eb in (("src_code_lo", 2), ("src_code_hi", 1), ("dst_w", 8)):
        base = lay[name][0]
        _hip_copy_d2d(base + a * eb, base, m * eb)
    with pytest.raises(_lib.AbnnError, match="tally and the records disagree; the records are not valid"):
        g.encode_traversal(1)
    refused()
    reload()

    for k in range(3):  # reloaded: the passes run and equal the oracle's
        g.encode_traversal(1)
        o.pass_serial()
        _same(g, o, f"after reload, pass {k}")
