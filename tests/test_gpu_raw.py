"""GPU parity of the buffer-index launcher (abnn_launch_traversal /
abnn_launch_renormalise): the reference kernel's 14 buffers (brain.metal:42-58)
as caller-owned device memory in the reference's own layouts -- 16-B
SynapsePacked records, u32 lastF / clock / budget -- against the CPU oracle,
bit-exact, pass by pass.  Device memory comes from torch (plumbing); every pass
runs through the C-ABI.  The host side of each pass restates
Brain::encode_traversal (brain.cpp:87-122): budget = kMaxSpikes, then one
dispatch; inputs are stamped `now` by the host before it (inject_inputs with
every input firing, brain.cpp:73-83)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=[0, 1], ids=["five_launches", "fused"])
def raw_pass_kind(request):
    """Every test runs both buffer-index passes: the five-launch one and the
    single k_raw_pass launch after the filter (abnn_debug_raw_fused)."""
    from abnn_amd import _lib

    lib = _lib.load()
    assert lib.abnn_debug_raw_fused(request.param) == 0
    yield request.param
    lib.abnn_debug_raw_fused(-1)


class RawBrain:
    """Caller-owned buffers, as Brain::build_buffers allocates them (brain.cpp:52-69)."""

    def __init__(self, syn: np.ndarray, n_nrn: int, events: int, max_spikes: int = 2560, knobs=None,
                 pool_chunks=None, ws=None):
        import torch

        from abnn_amd import _lib

        self.lib = _lib.load()
        self.t = torch
        dev = torch.device("cuda", 0)
        self.syn = torch.from_numpy(syn.view(np.uint32).reshape(-1, 4).copy()).to(dev)
        self.lastF = torch.zeros(n_nrn, dtype=torch.int32, device=dev)
        self.lastV = torch.zeros(n_nrn, dtype=torch.int32, device=dev)
        self.scal = torch.zeros(4, dtype=torch.int32, device=dev)  # clock, budget, reward, rBar
        self.n_syn, self.n_nrn, self.events, self.max_spikes = syn.shape[0], n_nrn, events, max_spikes
        # pool_chunks: None = the recommended workspace, else the least one plus
        # that many 4-KiB survivor chunks (0: every survivor recomputed)
        nb = int(self.lib.abnn_traversal_workspace_bytes(self.n_syn, events)) if pool_chunks is None else \
            int(self.lib.abnn_traversal_workspace_min_bytes(self.n_syn, events)) + 4096 * pool_chunks
        if ws is not None:  # another brain's workspace (at least as large)
            assert ws.numel() >= nb
            nb = ws.numel()
        self.ws = torch.zeros(max(16, nb), dtype=torch.uint8, device=dev) if ws is None else ws
        self.knobs = knobs
        a = _lib.TraversalArgs()
        p = self.scal.data_ptr()
        a.syn, a.last_fired, a.last_visited, a.clock = self.syn.data_ptr(), self.lastF.data_ptr(), \
            self.lastV.data_ptr(), p
        a.n_syn, a.tau_vis, a.tau_pre = self.n_syn, 50_000, 50_000
        kp = knobs if knobs is not None else _lib.default_params()
        a.a_ltp, a.a_ltd, a.w_min, a.w_max = kp.a_ltp, kp.a_ltd, kp.w_min, kp.w_max
        a.budget, a.reward, a.rbar = p + 4, p + 8, p + 12
        a.n_nrn, a.events = n_nrn, events
        a.knobs = C.cast(C.pointer(knobs), C.c_void_p) if knobs is not None else None
        a.workspace, a.workspace_bytes = self.ws.data_ptr(), nb
        self.args = a

    def pass_stats(self) -> tuple[int, int]:
        """The last pass's {pre-gated, refractory survivors} (abnn_debug_raw_stats)."""
        g = (C.c_uint64 * 2)()
        assert self.lib.abnn_debug_raw_stats(self.ws.data_ptr(), g, None) == 0
        return int(g[0]), int(g[1])

    def workspace_error(self) -> int:
        e = C.c_uint32(7)
        assert self.lib.abnn_traversal_workspace_error(self.ws.data_ptr(), C.byref(e), None) == 0
        return int(e.value)

    def set_clock(self, v: int) -> None:
        self.scal[0] = np.int32(np.uint32(v).view(np.int32))

    def set_reward(self, r: float) -> None:
        self.scal[2] = int(np.float32(r).view(np.int32))

    def one_pass(self, stim: int = 256) -> None:
        t = self.t
        if stim:  # inject_inputs with every input firing: lastF[i] = clock (brain.cpp:82)
            self.lastF[:stim] = self.scal[0]
        self.scal[1] = self.max_spikes  # encode_traversal resets the budget (brain.cpp:90)
        assert self.lib.abnn_launch_traversal(C.byref(self.args), None) == 0
        t.cuda.synchronize()

    def renormalise(self) -> None:
        assert self.lib.abnn_launch_renormalise(self.lastF.data_ptr(), self.lastV.data_ptr(), self.scal.data_ptr(),
                                                self.n_nrn, None) == 0
        self.t.cuda.synchronize()

    def records(self) -> np.ndarray:
        return self.syn.cpu().numpy().reshape(-1).view(np.uint32)

    def last_fired(self) -> np.ndarray:
        return self.lastF.cpu().numpy().view(np.uint32)

    def scalars(self):
        s = self.scal.cpu().numpy()
        return int(s[0].view(np.uint32)), int(s[1].view(np.uint32)), float(s[3].view(np.float32))


def _run(n_hidden, n_syn, events, passes, seed=1, max_spikes=2560, reward_at=None, tombstones=0, renorm_at=None,
         clock0=0, knobs=None, pool_chunks=None, threads=0):
    from oracle import oracle as O

    n_nrn = 512 + n_hidden
    over = {} if knobs is None else {k: getattr(knobs, k) for k, _ in O.Params._fields_}
    over["max_spikes"] = max_spikes
    over["renorm_thresh"] = 2**64 - 1  # the raw launcher's host decides renormalisation (renorm_at below)
    o = O.OracleBrain(256, 256, n_hidden, n_syn, events, **over)
    o.build_random_graph(seed, nthreads=max(8, threads))
    if tombstones:  # pruned records {0xFFFFFFFF, 0xFFFFFFFF} (abnn.h): never pass
        idx = np.arange(0, n_syn, max(1, n_syn // tombstones))[:tombstones]
        s = o.syn.copy()
        s["src"][idx] = 0xFFFFFFFF
        s["dst"][idx] = 0xFFFFFFFF
        o.set_synapses(s)
    o.set_scalars(clock0, 0.0, 0.0)
    r = RawBrain(o.syn.copy(), n_nrn, events, max_spikes, knobs, pool_chunks)
    r.set_clock(clock0)
    for k in range(passes):
        if reward_at is not None and k == reward_at:
            o.set_reward(0.5)
            r.set_reward(0.5)
        o.set_timestamps(range(256), o.clock)
        before = o.stats()["fired"]
        st0 = o.stats()
        if threads:
            o.pass_threaded(1, nthreads=threads)
        else:
            o.pass_serial()
        r.one_pass()
        if renorm_at is not None and k == renorm_at:  # the host's decision (brain.cpp:127-128)
            base = o.clock
            o.last_fired[:] = (o.last_fired - np.uint64(base)) & np.uint64(0xFFFFFFFF)
            o.set_scalars(0, o.s.reward, o.s.rbar)
            r.renormalise()
        clock, budget, rbar = r.scalars()
        assert clock == o.clock & 0xFFFFFFFF, k
        assert budget == max_spikes - (o.stats()["fired"] - before), k
        assert np.float32(rbar) == np.float32(o.s.rbar), k
        assert np.array_equal(r.last_fired(), (o.last_fired & np.uint64(0xFFFFFFFF)).astype(np.uint32)), k
        assert np.array_equal(r.records(), o.syn.view(np.uint32)), k
        assert r.workspace_error() == 0, k
        st1 = o.stats()
        assert r.pass_stats() == (st1["pre_gated"] - st0["pre_gated"], st1["post_gated"] - st0["post_gated"]), k
    return o


def test_raw_config1_every_pass(gpu):
    o = _run(488, 10_000, 100_000, 40, reward_at=15)  # BASELINE configs[0]
    assert o.stats()["fired"] > 0


def test_raw_c2lite_budget_saturated(gpu):
    # 100k neurons, 1M synapses: all-gated passes 3-5, then the budget-saturated steady state
    o = _run(99_488, 1_000_000, 1_000_000, 14, reward_at=7)
    st = o.stats()
    assert st["fired"] >= 2560 * 4 and st["updated"] > st["fired"]


@pytest.mark.parametrize("max_spikes", [0, 1, 37, 10**8])
def test_raw_budgets(gpu, max_spikes):
    _run(9_488, 200_000, 150_000, 8, max_spikes=max_spikes)


def test_raw_partial_sweep_tombstones_and_odd_events(gpu):
    # events not a multiple of 256 (grid rounds up, brain.cpp:116-118), fewer
    # records than the grid for one, tombstoned records
    _run(9_488, 100_000, 54_321, 8, tombstones=500)
    _run(9_488, 3_000, 4_097, 8)


def test_raw_renormalise_and_clock_near_wrap(gpu):
    _run(9_488, 100_000, 100_000, 10, renorm_at=6, clock0=3_999_990)
    _run(9_488, 100_000, 100_000, 8, clock0=0xFFFFFFFF - 3)  # u32 clock wraps mid-run (brain.metal:45)


def test_raw_knobs(gpu):
    from abnn_amd import _lib

    k = _lib.default_params(base_scale=1.7, refractory=0, window_pre=2, eta_home=1e-4, a_ltp=0.08, w_min=0.05)
    _run(9_488, 100_000, 100_000, 8, knobs=k, reward_at=2)


@pytest.mark.parametrize("pool_chunks", [0, 3, 4200])
def test_raw_survivor_pool_overflow_recomputes(gpu, pool_chunks):
    """Survivors that do not fit the bounded pool (none, a few chunks, one
    chunk per gate wave and some) are recomputed from the records by
    k_raw_apply with the pass-start lastF: the same results, the all-gated
    passes 3-5 of a fresh graph included."""
    o = _run(99_488, 1_000_000, 1_000_000, 10, reward_at=5, pool_chunks=pool_chunks)
    assert o.stats()["post_gated"] > 1_000_000  # the transient overflowed every pool tried


def test_raw_direct_stamps_with_pool_overflow_are_reported(gpu):
    """A pass whose spikes exceed the spike list (min(E, 65536) entries; an
    unbounded budget) stamps directly; with survivors recomputed as well,
    abnn_traversal_workspace_error says so (abnn.h).  Config 2's 10M events:
    the all-gated passes 3-5 emit ~10^5 spikes each."""
    from oracle import oracle as O

    n = 10_000_000
    o = O.OracleBrain(256, 256, 99_488, n, n)
    o.build_random_graph(1, nthreads=16)
    r = RawBrain(o.syn.copy(), 100_000, n, 10**8, pool_chunks=0)
    for _ in range(5):  # passes 3-5: every event gated, candidates far beyond the budget list
        r.one_pass()
    assert r.workspace_error() == 1  # sticky: set in passes 3-5, still seen after pass 5
    assert r.workspace_error() == 0  # ... and cleared by the read


def test_raw_budget_above_list_with_pool_overflow_is_exact(gpu):
    """A budget above the spike list does not by itself stamp directly: only a
    pass whose spikes exceed the list does.  With E <= 65536 the
    list holds every spike, so even with every survivor recomputed (no pool)
    and an unbounded budget the stamps wait for the last lastF read: exact,
    no error."""
    _run(9_488, 200_000, 60_000, 8, max_spikes=10**8, pool_chunks=0)


def test_raw_config3_bit_exact_vs_threaded_oracle(gpu):
    """The reference layout at config 3 (5,000,512 neurons; 150,000,128
    visited events: the first records of the 1B graph, the only ones a sweep
    reads): 16 passes from the fresh graph through its all-gated transient
    into the budget-saturated steady state, every pass bit-exact against the
    threaded oracle -- records, u32 lastF, clock, budget left, rBar."""
    o = _run(5_000_000, 150_000_128, 150_000_000, 16, reward_at=9, threads=32)
    st = o.stats()
    assert st["fired"] >= 2560 * 8 and st["updated"] > st["fired"]


def test_raw_workspace_reused_across_sizes(gpu):
    """One workspace for passes of different n_syn / events, interleaved
    (ADVICE r5): the state the fused pass keeps across passes (epoch-tagged
    look-back words, bounds, costs) lives at offsets that do not depend on E,
    so a pass of another size never reads a spike list or a bound of the
    other as a published look-back word.  Every pass bit-exact against its
    oracle."""
    from oracle import oracle as O

    sizes = [(99_488, 1_000_000, 1_000_000), (9_488, 200_000, 150_000), (9_488, 3_000, 4_097)]
    pairs, ws = [], None
    for n_hidden, n_syn, events in sizes:
        o = O.OracleBrain(256, 256, n_hidden, n_syn, events, renorm_thresh=2**64 - 1)
        o.build_random_graph(3, nthreads=8)
        o.set_scalars(0, 0.0, 0.0)
        r = RawBrain(o.syn.copy(), 512 + n_hidden, events, ws=ws)
        ws = r.ws if ws is None else ws  # the first (largest) workspace serves all three
        pairs.append((o, r))
    for k in range(18):
        o, r = pairs[(k // 2) % 3]  # two passes each, round robin: every switch changes E
        o.set_timestamps(range(256), o.clock)
        o.pass_serial()
        r.one_pass()
        clock, _, rbar = r.scalars()
        assert clock == o.clock & 0xFFFFFFFF, k
        assert np.float32(rbar) == np.float32(o.s.rbar), k
        assert np.array_equal(r.last_fired(), (o.last_fired & np.uint64(0xFFFFFFFF)).astype(np.uint32)), k
        assert np.array_equal(r.records(), o.syn.view(np.uint32)), k
        assert r.workspace_error() == 0, k
