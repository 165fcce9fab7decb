"""ctypes wrapper of the C oracle (c1_oracle.c).

TEST INFRASTRUCTURE ONLY: may be imported by tests/, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of bench.py -- never by the product (abnn_amd/).
PARITY UNPINNED: see c1_oracle.h and DESIGN.md §3.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")

SYN_DTYPE = np.dtype([("src", "<u4"), ("dst", "<u4"), ("w", "<f4"), ("pad", "<f4")])
G2_DTYPE = np.dtype([("t", "<u8"), ("isi", "<f4"), ("pre", "<u4"), ("cand", "<u4"), ("w", "<f4")])
SUMMARY_WORDS = 4


class Dims(C.Structure):
    _fields_ = [("n_input", C.c_uint32), ("n_output", C.c_uint32), ("n_hidden", C.c_uint64),
                ("n_syn", C.c_uint64), ("events_per_pass", C.c_uint64),
                ("syn_offset", C.c_uint64), ("global_events", C.c_uint64),
                ("syn_capacity", C.c_uint64)]


class Params(C.Structure):
    _fields_ = [("base_scale", C.c_float), ("refractory", C.c_uint32),
                ("window_pre", C.c_uint32), ("clock_inc", C.c_uint32),
                ("target_rate_hz", C.c_float), ("eta_home", C.c_float),
                ("eta_reward", C.c_float), ("alpha_rbar", C.c_float), ("a_ltp", C.c_float),
                ("a_ltd", C.c_float), ("w_min", C.c_float), ("w_max", C.c_float),
                ("max_spikes", C.c_uint32), ("tick_ns", C.c_uint32), ("tau_vis", C.c_uint32),
                ("tau_pre", C.c_uint32), ("renorm_thresh", C.c_uint64),
                ("track_visits", C.c_uint32), ("mode", C.c_uint32), ("seed", C.c_uint64),
                ("w_prune", C.c_float), ("p_new", C.c_float), ("w_init", C.c_float),
                ("compact_every", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("passes", C.c_uint64), ("events", C.c_uint64), ("pre_gated", C.c_uint64),
                ("post_gated", C.c_uint64), ("updated", C.c_uint64), ("fired", C.c_uint64),
                ("pruned", C.c_uint64), ("grown", C.c_uint64)]


class State(C.Structure):
    _fields_ = [("dims", Dims), ("p", Params), ("n_nrn", C.c_uint64), ("syn", C.c_void_p),
                ("last_fired", C.c_void_p), ("last_visited", C.c_void_p), ("clock", C.c_uint64),
                ("reward", C.c_float), ("rbar", C.c_float), ("rng", C.c_uint64),
                ("stim_first", C.c_uint64), ("stim_count", C.c_uint64), ("stats", Stats),
                ("pass_index", C.c_uint64), ("grown", C.c_void_p), ("visit_mark", C.c_void_p),
                ("renorms", C.c_uint64)]


_lib = None


def load() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            import sys
            sys.path.insert(0, os.path.dirname(_HERE))
            from abnn_amd.build import build_oracle
            build_oracle()
        lib = C.CDLL(LIB_PATH)
        vp, u32, u64 = C.c_void_p, C.c_uint32, C.c_uint64
        sigs = {
            "oracle_default_params": (None, [C.POINTER(Params)]),
            "oracle_rand01": (C.c_float, [u32]),
            "oracle_splitmix64_at": (u64, [u64, u64]),
            "oracle_visited_events": (u64, [C.POINTER(Dims), u32]),
            "oracle_philox4x32_10": (None, [vp, vp, vp]),
            "oracle_pick": (u64, [u64, u64, u64, u64, u64]),
            "oracle_gen_synapses": (None, [vp, u64, u64, u32, u32, u64, u64, C.c_int]),
            "oracle_checksum_synapses": (u64, [vp, u64, u64]),
            "oracle_inject_inputs": (None, [C.POINTER(State), vp, u32, C.c_float]),
            "oracle_read_outputs": (None, [C.POINTER(State), vp, u32]),
            "oracle_pass_serial": (None, [C.POINTER(State)]),
            "oracle_pass_threaded": (None, [C.POINTER(State), C.c_int]),
            "oracle_exchange_words": (u32, [u32]),
            "oracle_shard_gate": (C.c_int64, [C.POINTER(State), vp, u64, vp]),
            "oracle_shard_apply": (None, [C.POINTER(State), vp, C.c_int64, vp, u32, u32]),
            "oracle_shard_commit": (None, [C.POINTER(State), vp, u32]),
        }
        for name, (res, args) in sigs.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _lib = lib
    return _lib


def default_params(**overrides) -> Params:
    p = Params()
    load().oracle_default_params(C.byref(p))
    for k, v in overrides.items():
        if not hasattr(p, k):
            raise KeyError(k)
        setattr(p, k, v)
    return p


def rand01(s: int) -> float:
    return float(load().oracle_rand01(s & 0xFFFFFFFF))


def gen_synapses(first: int, n: int, n_input: int, n_output: int, n_neuron: int, seed: int = 1,
                 nthreads: int = 1) -> np.ndarray:
    out = np.empty(n, dtype=SYN_DTYPE)
    load().oracle_gen_synapses(out.ctypes.data, first, n, n_input, n_output, n_neuron, seed,
                               nthreads)
    return out


def checksum(syn: np.ndarray, first_global: int = 0) -> int:
    syn = np.ascontiguousarray(syn, dtype=SYN_DTYPE)
    return int(load().oracle_checksum_synapses(syn.ctypes.data, syn.shape[0], first_global))


def visited_events(events: int, n_syn: int, mode: int = 0) -> int:
    d = Dims(0, 0, 0, n_syn, events, 0, 0)
    return int(load().oracle_visited_events(C.byref(d), mode))


def philox4x32_10(ctr, key) -> list[int]:
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    load().oracle_philox4x32_10(c, k, o)
    return list(o)


def pick(seed: int, stream: int, pass_index: int, t: int, n_syn: int) -> int:
    return int(load().oracle_pick(seed, stream, pass_index, t, n_syn))


class OracleBrain:
    """CPU C1 state with the same surface as abnn_amd.Brain (subset)."""

    def __init__(self, n_input: int, n_output: int, n_hidden: int, n_syn: int,
                 events_per_pass: int, *, syn_offset: int = 0, global_events: int = 0,
                 syn_capacity: int = 0, params: Optional[Params] = None, **param_overrides):
        self._lib = load()
        self.p = params if params is not None else default_params(**param_overrides)
        n_nrn = n_input + n_output + n_hidden
        cap = max(int(syn_capacity), int(n_syn))  # 0 = the creation size (as the C-ABI)
        self._syn = np.zeros(cap, dtype=SYN_DTYPE)
        self.last_fired = np.zeros(n_nrn, dtype=np.uint64)
        self.last_visited = np.zeros(n_nrn, dtype=np.uint64)
        self._grown = np.zeros(max(1, self.p.compact_every * self.p.max_spikes), dtype=SYN_DTYPE)
        # a shard that tracks visits marks them for the lastVisited merge (abnn.h)
        self.visit_mark = np.zeros(n_nrn, dtype=np.uint8) if (global_events and self.p.track_visits) else None
        self.s = State()
        self.s.dims = Dims(n_input, n_output, n_hidden, n_syn, events_per_pass, syn_offset,
                           global_events, cap)
        self.s.p = self.p
        self.s.n_nrn = n_nrn
        self.s.rng = self.p.seed
        self._bind()

    @property
    def syn(self) -> np.ndarray:
        """The current records (n_syn changes at structural updates)."""
        return self._syn[: int(self.s.dims.n_syn)]

    def _bind(self) -> None:
        self.s.syn = self._syn.ctypes.data
        self.s.last_fired = self.last_fired.ctypes.data
        self.s.last_visited = self.last_visited.ctypes.data
        self.s.grown = self._grown.ctypes.data
        self.s.visit_mark = self.visit_mark.ctypes.data if self.visit_mark is not None else None

    # state ---------------------------------------------------------------------------------
    def n_neuron(self) -> int:
        return int(self.s.n_nrn)

    def build_random_graph(self, seed: int = 1, nthreads: int = 8) -> None:
        d = self.s.dims
        self._lib.oracle_gen_synapses(self.syn.ctypes.data, d.syn_offset, d.n_syn, d.n_input,
                                      d.n_output, self.s.n_nrn, seed, nthreads)

    def set_synapses(self, syn: np.ndarray) -> None:
        self._syn[: syn.shape[0]] = syn

    def checksum(self) -> int:
        return checksum(self.syn, int(self.s.dims.syn_offset))

    def scalars(self) -> dict:
        return {"clock": int(self.s.clock), "reward": float(self.s.reward), "rbar": float(self.s.rbar),
                "pass_index": int(self.s.pass_index)}

    def set_scalars(self, clock: int, reward: float, rbar: float, pass_index: Optional[int] = None) -> None:
        self.s.clock, self.s.reward, self.s.rbar = clock, reward, rbar
        if pass_index is not None:
            self.s.pass_index = pass_index

    def set_reward(self, r: float) -> None:
        self.s.reward = r

    def set_timestamps(self, idx: Sequence[int], value: int) -> None:
        self.last_fired[np.asarray(idx, dtype=np.int64)] = np.uint64(value)

    def set_last_visited(self, values, first: int = 0) -> None:
        """Host write (replicated on every shard): replaces what this shard
        visited before it (abnn_set_last_visited clears those marks)."""
        v = np.asarray(values, dtype=np.uint64)
        self.last_visited[first:first + v.shape[0]] = v
        if self.visit_mark is not None:
            self.visit_mark[first:first + v.shape[0]] = 0

    def renormalisations(self) -> int:
        return int(self.s.renorms)

    def visits_delta(self) -> np.ndarray:
        """abnn_shard_visits_delta restated: visited ? lastVisited + 1 : 0 (int64 view)."""
        if self.visit_mark is None:
            return np.zeros(self.last_visited.shape[0], dtype=np.int64)
        d = np.where(self.visit_mark != 0, self.last_visited + np.uint64(1), np.uint64(0))
        return d.view(np.int64)

    def visits_merge(self, reduced: np.ndarray) -> None:
        """abnn_shard_visits_merge restated."""
        r = np.asarray(reduced).view(np.uint64)
        nz = r != 0
        self.last_visited[nz] = r[nz] - np.uint64(1)
        if self.visit_mark is not None:
            self.visit_mark[:] = 0

    def set_auto_stimulus(self, first: int, count: int) -> None:
        self.s.stim_first, self.s.stim_count = first, count

    def inject_inputs(self, vals: Sequence[float], hz: float) -> None:
        v = np.ascontiguousarray(vals, dtype=np.float32)
        self._lib.oracle_inject_inputs(C.byref(self.s), v.ctypes.data, v.shape[0], hz)

    def read_outputs(self) -> np.ndarray:
        out = np.zeros(self.s.dims.n_output, dtype=np.uint8)
        self._lib.oracle_read_outputs(C.byref(self.s), out.ctypes.data, out.shape[0])
        return out.astype(bool)

    def stats(self) -> dict:
        st = self.s.stats
        return {k: int(getattr(st, k)) for k, _ in Stats._fields_}

    # passes --------------------------------------------------------------------------------
    def pass_serial(self, passes: int = 1) -> None:
        for _ in range(passes):
            self._lib.oracle_pass_serial(C.byref(self.s))

    def pass_threaded(self, passes: int = 1, nthreads: int = 8) -> None:
        for _ in range(passes):
            self._lib.oracle_pass_threaded(C.byref(self.s), nthreads)

    # shard phases (one exchange: include/abnn/abnn.h) ------------------------------------
    def exchange_words(self) -> int:
        """int32 words of one shard's exchange record (summary + local spike list)."""
        return int(self._lib.oracle_exchange_words(self.p.max_spikes))

    def shard_gate(self, xchg: np.ndarray) -> np.ndarray:
        """Gate phase; writes this shard's record into `xchg` (int32, exchange_words())."""
        assert xchg.dtype == np.int32 and xchg.shape[0] >= self.exchange_words()
        ev = visited_events(int(self.s.dims.events_per_pass), int(self.s.dims.n_syn), int(self.p.mode))
        buf = np.zeros(max(1, ev), dtype=G2_DTYPE)
        n = self._lib.oracle_shard_gate(C.byref(self.s), buf.ctypes.data, buf.shape[0], xchg.ctypes.data)
        if n < 0:
            raise RuntimeError("oracle_shard_gate overflow")
        self._g2 = buf[:n].copy()
        return self._g2

    def shard_apply(self, gathered: np.ndarray, world: int, rank: int) -> None:
        self._lib.oracle_shard_apply(C.byref(self.s), self._g2.ctypes.data, self._g2.shape[0],
                                     gathered.ctypes.data, world, rank)

    def shard_commit(self, gathered: np.ndarray, world: int) -> None:
        self._lib.oracle_shard_commit(C.byref(self.s), gathered.ctypes.data, world)

    @property
    def clock(self) -> int:
        return int(self.s.clock)
