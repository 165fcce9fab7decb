"""Python mirror of the reference host class ``Brain`` over the C-ABI.

Reference: abnn/src/core/brain/brain.h:24-83 and brain.cpp:21-178.  Method
names follow the reference (``encode_traversal``, ``inject_inputs``,
``read_outputs``, ``save``/``load``, ``n_input()`` ...); Metal types are
replaced by the HIP engine behind ``libabnn_hip.so``.  All compute runs in the
HIP library -- this module only moves small host arrays and pointers.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import Dims, Params, Scalars, State, Stats, call

# SynapsePacked {u32 src, u32 dst, f32 w, f32 pad} (brain.metal:11, brain.h:21)
SYN_DTYPE = np.dtype([("src", "<u4"), ("dst", "<u4"), ("w", "<f4"), ("pad", "<f4")])


def visited_events(events_per_pass: int, n_syn: int, mode: int = 0) -> int:
    """Sweep: min(roundup(EVENTS,256), nSyn) -- brain.cpp:116-118 with
    brain.metal:60-61.  Random mode: exactly EVENTS picks (README §4)."""
    if mode == _lib.MODE_RANDOM:
        return int(events_per_pass) if int(n_syn) else 0
    grid = (int(events_per_pass) + 255) // 256 * 256
    return min(grid, int(n_syn))


def _stream_ptr(stream) -> Optional[int]:
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return int(getattr(stream, "cuda_stream"))  # torch.cuda.Stream


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class Brain:
    """One traversal engine on one GPU (optionally one synapse shard)."""

    def __init__(self, n_input: int, n_output: int, n_hidden: int, n_syn: int,
                 events_per_pass: int, *, params: Optional[Params] = None, device: int = 0,
                 syn_offset: int = 0, global_events: int = 0, syn_capacity: int = 0,
                 **param_overrides):
        self._lib = _lib.load()
        if params is None:
            params = _lib.default_params(**param_overrides)
        elif param_overrides:
            raise TypeError("pass either params= or keyword overrides, not both")
        self._dims = Dims(n_input, n_output, n_hidden, n_syn, events_per_pass, syn_offset,
                          global_events, syn_capacity)
        self._params = params
        h = C.c_void_p()
        call("abnn_brain_create", C.byref(self._dims), C.byref(params), int(device), C.byref(h))
        self._h = h
        self.device = int(device)

    # ---- lifetime -------------------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            call("abnn_brain_destroy", self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- getters (brain.h:48-52) --------------------------------------------------------------
    def n_input(self) -> int:
        return int(self._dims.n_input)

    def n_output(self) -> int:
        return int(self._dims.n_output)

    def n_hidden(self) -> int:
        return int(self._dims.n_hidden)

    def n_neuron(self) -> int:
        return int(self._lib.abnn_n_neuron(self._h))

    def n_syn(self) -> int:
        """Current record count (structural updates change it)."""
        return int(self.dims.n_syn)

    @property
    def dims(self) -> Dims:
        d = Dims()
        call("abnn_get_dims", self._h, C.byref(d))
        return d

    @property
    def params(self) -> Params:
        return self._params

    def visited_events(self) -> int:
        return visited_events(self._dims.events_per_pass, self.n_syn(), self._params.mode)

    def state_ptrs(self) -> dict:
        """Borrowed device pointers (brain.h:54-58); ``synapses`` is opaque."""
        s = State()
        call("abnn_state_ptrs", self._h, C.byref(s))
        return {k: int(getattr(s, k) or 0) for k, _ in State._fields_}

    def synapse_layout(self) -> dict:
        """The device record layout behind state_ptrs()['synapses'] (versioned apart from the ABI)."""
        lay = _lib.Layout()
        call("abnn_synapse_layout", self._h, C.byref(lay))
        arrays = {lay.arrays[i].name.decode(): (int(lay.arrays[i].ptr or 0), int(lay.arrays[i].bytes),
                                                int(lay.arrays[i].elem_bytes)) for i in range(lay.n_arrays)}
        return {"version": int(lay.version), "arrays": arrays}

    def budget(self) -> int:
        """Spike budget left by the last pass (bufBudget_, brain.h:58)."""
        v = C.c_uint32()
        call("abnn_get_budget", self._h, C.byref(v))
        return int(v.value)

    def structural_updates(self) -> int:
        """Structural updates run so far (host count, no synchronisation)."""
        return int(self._lib.abnn_structural_updates(self._h))

    def renormalisations(self) -> int:
        """Renormalisations run so far (host count, no synchronisation)."""
        return int(self._lib.abnn_renormalisations(self._h))

    # ---- synapses ------------------------------------------------------------------------------
    def upload_synapses(self, syn: np.ndarray, first: int = 0) -> None:
        syn = np.ascontiguousarray(syn, dtype=SYN_DTYPE)
        call("abnn_upload_synapses", self._h, first, _ptr(syn), syn.shape[0])

    def download_synapses(self, first: int = 0, n: Optional[int] = None) -> np.ndarray:
        n = self.n_syn() - first if n is None else n
        out = np.empty(n, dtype=SYN_DTYPE)
        call("abnn_download_synapses", self._h, first, _ptr(out), n)
        return out

    def build_random_graph(self, seed: int = 1) -> None:
        """build_random_graph recipe (brain-engine.cpp:31-53), generated on the GPU."""
        call("abnn_generate_synapses", self._h, seed)

    def checksum(self) -> int:
        v = C.c_uint64()
        call("abnn_checksum_synapses", self._h, C.byref(v))
        return int(v.value)

    # ---- neuron state ---------------------------------------------------------------------------
    def last_fired(self, first: int = 0, n: Optional[int] = None) -> np.ndarray:
        n = self.n_neuron() - first if n is None else n
        out = np.empty(n, dtype=np.uint64)
        call("abnn_get_last_fired", self._h, first, _ptr(out), n)
        return out

    def set_last_fired(self, values: np.ndarray, first: int = 0) -> None:
        v = np.ascontiguousarray(values, dtype=np.uint64)
        call("abnn_set_last_fired", self._h, first, _ptr(v), v.shape[0])

    def last_visited(self, first: int = 0, n: Optional[int] = None) -> np.ndarray:
        n = self.n_neuron() - first if n is None else n
        out = np.empty(n, dtype=np.uint64)
        call("abnn_get_last_visited", self._h, first, _ptr(out), n)
        return out

    def set_last_visited(self, values: np.ndarray, first: int = 0) -> None:
        v = np.ascontiguousarray(values, dtype=np.uint64)
        call("abnn_set_last_visited", self._h, first, _ptr(v), v.shape[0])

    def set_timestamps(self, idx: Sequence[int], value: int) -> None:
        i = np.ascontiguousarray(idx, dtype=np.uint32)
        call("abnn_set_timestamps", self._h, _ptr(i), i.shape[0], int(value))

    def scalars(self) -> dict:
        s = Scalars()
        call("abnn_get_scalars", self._h, C.byref(s))
        return {"clock": int(s.clock), "reward": float(s.reward), "rbar": float(s.rbar),
                "pass_index": int(s.pass_index)}

    def set_scalars(self, clock: int, reward: float, rbar: float, pass_index: Optional[int] = None) -> None:
        if pass_index is None:
            pass_index = self.scalars()["pass_index"]
        s = Scalars(clock, reward, rbar, pass_index)
        call("abnn_set_scalars", self._h, C.byref(s))

    def set_reward(self, r: float) -> None:
        call("abnn_set_reward", self._h, float(r))

    # ---- pass-boundary hooks ------------------------------------------------------------------
    def inject_inputs(self, vals: Sequence[float], hz: float) -> None:
        """Brain::inject_inputs (brain.cpp:73-83)."""
        v = np.ascontiguousarray(vals, dtype=np.float32)
        call("abnn_inject_inputs", self._h, _ptr(v), v.shape[0], float(hz))

    def read_outputs(self) -> np.ndarray:
        """Brain::read_outputs (brain.cpp:145-157) -> bool[n_output]."""
        out = np.zeros(self.n_output(), dtype=np.uint8)
        call("abnn_read_outputs", self._h, _ptr(out), out.shape[0])
        return out.astype(bool)

    def set_auto_stimulus(self, first: int, count: int) -> None:
        call("abnn_set_auto_stimulus", self._h, int(first), int(count))

    # ---- passes --------------------------------------------------------------------------------
    def encode_traversal(self, passes: int = 1, stream=None) -> None:
        """Brain::encode_traversal + commit (brain.cpp:87-141): enqueue whole C1 passes."""
        call("abnn_traverse", self._h, int(passes), _stream_ptr(stream))

    traverse = encode_traversal

    def synchronize(self, stream=None) -> None:
        call("abnn_synchronize", self._h, _stream_ptr(stream))

    def exchange_bytes(self) -> int:
        """Bytes of this shard's exchange record (summary + local spike list, abnn.h)."""
        return int(self._lib.abnn_exchange_bytes(self._h))

    def set_global_events(self, n: int) -> None:
        """Visited events of all shards per pass (after structural updates)."""
        call("abnn_set_global_events", self._h, int(n))

    def shard_gate(self, xchg_ptr: int, stream=None) -> None:
        call("abnn_shard_gate", self._h, xchg_ptr, _stream_ptr(stream))

    def shard_apply(self, gathered_ptr: int, world: int, rank: int, stream=None) -> None:
        call("abnn_shard_apply", self._h, gathered_ptr, world, rank, _stream_ptr(stream))

    def shard_commit(self, gathered_ptr: int, world: int, stream=None) -> None:
        call("abnn_shard_commit", self._h, gathered_ptr, world, _stream_ptr(stream))

    def shard_visits_delta(self, delta_ptr: int, stream=None) -> None:
        """This shard's lastVisited merge deltas (u64 x N_NRN, device; abnn.h)."""
        call("abnn_shard_visits_delta", self._h, delta_ptr, _stream_ptr(stream))

    def shard_visits_merge(self, reduced_ptr: int, stream=None) -> None:
        """Apply the all-reduced (MAX) deltas; clears this shard's visit marks."""
        call("abnn_shard_visits_merge", self._h, reduced_ptr, _stream_ptr(stream))

    # ---- statistics / timing ------------------------------------------------------------------
    def stats(self) -> dict:
        s = Stats()
        call("abnn_get_stats", self._h, C.byref(s))
        return s.as_dict()

    def reset_stats(self) -> None:
        call("abnn_reset_stats", self._h)

    def enable_timing(self, on: bool | int = True) -> None:
        """True/1: time every gate launch; n > 1: every n-th; False/0: off."""
        call("abnn_enable_timing", self._h, int(on))

    def kernel_time(self) -> tuple[float, int]:
        ms = C.c_double()
        n = C.c_uint64()
        call("abnn_get_kernel_time", self._h, C.byref(ms), C.byref(n))
        return float(ms.value), int(n.value)

    def kernel_times(self, cap: int = 1 << 16) -> np.ndarray:
        """The timed gate launches since the last call, one by one (ms)."""
        out = np.zeros(cap, dtype=np.float32)
        n = C.c_uint64()
        call("abnn_get_kernel_times", self._h, _ptr(out), cap, C.byref(n))
        return out[:min(int(n.value), cap)].astype(np.float64)

    # ---- persistence (brain.cpp:161-178, README §2) --------------------------------------------
    def save(self, path: str | os.PathLike) -> None:
        call("abnn_save_bnn", self._h, os.fsencode(path))

    def load(self, path: str | os.PathLike) -> None:
        call("abnn_load_bnn", self._h, os.fsencode(path))

    def save_flat(self, path: str | os.PathLike) -> None:
        call("abnn_save_flat", self._h, os.fsencode(path))

    def load_flat(self, path: str | os.PathLike) -> None:
        call("abnn_load_flat", self._h, os.fsencode(path))
