"""Synapse-shard data parallelism: one process per GPU, exchange over RCCL.

The reference is single-GPU (no NCCL/MPI anywhere).  The build
shards the synapse array in contiguous ranges across ranks, replicates the
neuron state (lastFired, lastVisited, clock, reward, rBar) and keeps schedule
C1 bit-exact with ONE exchange per pass: after the gate phase
every rank all-gathers each rank's record (include/abnn/abnn.h) -- its
summary (4 x int64: spike candidates capped at the budget, global-event-0
flag, visited events, gated events) followed by its spikes in local budget
order (max_spikes x int32).  From the gathered records every rank knows its
offset in the ordered global spike budget (apply) and the global spike list
(rank order = budget order: commit stamps it).  All stamps of a pass write the
same value ``now``, so this equals the north-star all-reduce(MAX) over
lastFired exactly, at ~10 KB per rank instead of 40 MB per pass.

``lastVisited`` feeds no decision (brain.metal:44), so it is merged lazily
(:func:`merge_visits`): unsharded it holds the LAST value written, so each
shard contributes only the neurons it visited since the previous merge
(value + 1, else 0), the contributions are all-reduced with MAX, and a
non-zero result replaces the value everywhere.  MAX picks the last writer
because the clock only moves forward between merges: one is forced after
every renormalisation (:func:`sharded_pass`), and the C-ABI refuses to move
the clock back over unmerged visits.
"""
from __future__ import annotations

from typing import Protocol

import numpy as np

from .brain import Brain, visited_events


def shard_ranges(n_syn_global: int, world: int) -> list[tuple[int, int]]:
    """Contiguous, balanced [lo, hi) synapse ranges; rank order = global tid order."""
    base, extra = divmod(int(n_syn_global), int(world))
    out, lo = [], 0
    for r in range(world):
        hi = lo + base + (1 if r < extra else 0)
        out.append((lo, hi))
        lo = hi
    return out


def global_events(n_syn_global: int, events_per_pass: int, world: int, mode: int = 0) -> int:
    """Visited events per pass over all shards (each shard sweeps, or picks
    within, its own range)."""
    return sum(visited_events(events_per_pass, hi - lo, mode) for lo, hi in shard_ranges(n_syn_global, world))


class Engine(Protocol):
    """One shard's pass phases (the GPU Brain, or a CPU stand-in in tests)."""

    def gate(self, xchg) -> None: ...

    def apply(self, gathered, world: int, rank: int) -> None: ...

    def commit(self, gathered, world: int) -> None: ...

    def tracks_visits(self) -> bool: ...

    def renormalisations(self) -> int: ...

    def visits_delta(self):
        """int64 tensor of N_NRN merge deltas (abnn_shard_visits_delta)."""

    def visits_merge(self, reduced) -> None: ...


class TorchComm:
    """torch.distributed communicator.

    backend nccl (= RCCL on ROCm): the collectives run on device tensors, ordered
    with the pass kernels through the current stream.  backend gloo (CPU tests,
    or the single-GPU rehearsal of the multi-rank bench): device tensors are
    staged through host memory."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self._dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.staged = dist.get_backend(group) == "gloo"

    def _run(self, fn, *tensors):
        if not (self.staged and any(t.is_cuda for t in tensors)):
            fn(*tensors)
            return
        host = [t.cpu() for t in tensors]
        fn(*host)
        for t, h in zip(tensors, host):
            t.copy_(h)

    def all_gather(self, out, inp) -> None:
        self._run(lambda o, i: self._dist.all_gather_into_tensor(o, i, group=self.group), out, inp)

    def all_reduce_max(self, t) -> None:
        self._run(lambda x: self._dist.all_reduce(x, op=self._dist.ReduceOp.MAX, group=self.group), t)

    def all_reduce_sum(self, t) -> None:
        self._run(lambda x: self._dist.all_reduce(x, op=self._dist.ReduceOp.SUM, group=self.group), t)


def merge_visits(engine: Engine, comm) -> None:
    """The lastVisited merge (abnn.h abnn_shard_visits_delta / _merge): every
    rank's deltas, one all-reduce(MAX), the merge.  Collective: every rank
    calls it at the same point."""
    if not engine.tracks_visits():
        return
    delta = engine.visits_delta()
    comm.all_reduce_max(delta)
    engine.visits_merge(delta)


def sharded_pass(engine: Engine, comm, xchg, gathered) -> None:
    """One C1 pass over all shards: gate -> all-gather of the records -> apply
    -> commit; after a renormalisation (the clock went back) the lastVisited
    merge, before the next pass stamps values below this epoch's."""
    renorms = engine.renormalisations()
    engine.gate(xchg)
    comm.all_gather(gathered, xchg)
    engine.apply(gathered, comm.world, comm.rank)
    engine.commit(gathered, comm.world)
    if engine.renormalisations() != renorms:  # every rank renormalises after the same pass
        merge_visits(engine, comm)


class _GpuEngine:
    def __init__(self, brain: Brain, stream_fn):
        self.brain = brain
        self._stream = stream_fn

    def gate(self, xchg) -> None:
        self.brain.shard_gate(xchg.data_ptr(), self._stream())

    def apply(self, gathered, world, rank) -> None:
        self.brain.shard_apply(gathered.data_ptr(), world, rank, self._stream())

    def commit(self, gathered, world) -> None:
        self.brain.shard_commit(gathered.data_ptr(), world, self._stream())

    def tracks_visits(self) -> bool:
        return bool(self.brain.params.track_visits)

    def renormalisations(self) -> int:
        return self.brain.renormalisations()

    def visits_delta(self):
        import torch

        dev = torch.device("cuda", self.brain.device)
        t = torch.empty(self.brain.n_neuron(), dtype=torch.int64, device=dev)
        self.brain.shard_visits_delta(t.data_ptr(), self._stream())
        return t

    def visits_merge(self, reduced) -> None:
        self.brain.shard_visits_merge(reduced.data_ptr(), self._stream())


class NativeComm:
    """The library's own RCCL communicator (abnn_comm, include/abnn/abnn.h):
    rank 0's unique id is broadcast over ``torch.distributed`` once, then
    every pass's all-gather is enqueued by the C-ABI itself
    (abnn_shard_traverse) -- no Python, no torch collective per pass."""

    def __init__(self, device: int, group=None):
        import ctypes as C

        import torch
        import torch.distributed as dist

        from . import _lib

        self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)
        uid = np.zeros(_lib.COMM_ID_BYTES, dtype=np.uint8)
        if self.rank == 0:
            _lib.call("abnn_comm_unique_id", uid.ctypes.data)
        on_gpu = dist.get_backend(group) == "nccl"
        t = torch.from_numpy(uid).to(torch.device("cuda", device) if on_gpu else "cpu")
        src = dist.get_global_rank(group, 0) if group is not None else 0  # the group's rank 0
        dist.broadcast(t, src, group=group)
        uid = np.ascontiguousarray(t.cpu().numpy())
        h = C.c_void_p()
        _lib.call("abnn_comm_create", uid.ctypes.data, self.world, self.rank, int(device), C.byref(h))
        self.handle = h

    def close(self) -> None:
        from . import _lib

        if getattr(self, "handle", None) is not None and self.handle.value:
            _lib.call("abnn_comm_destroy", self.handle)
        self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class LocalGroup:
    """In-process communicator group (abnn_comm_group, include/abnn/abnn.h):
    ``world`` ranks in ONE process, one host thread per rank, each driving its
    shard handle through the C-ABI (abnn_shard_traverse) with the communicator
    :meth:`comm` returns.  The collectives are device copies and a reduction
    kernel between host barriers -- no RCCL: the sharded pass at world > 1 on
    one GPU (SURVEY §4 item 4's fake communicator behind the same interface).
    Ranks on one device must use one stream (torch's default stream in every
    thread does)."""

    def __init__(self, world: int):
        import ctypes as C

        from . import _lib

        self.world = int(world)
        h = C.c_void_p()
        _lib.call("abnn_comm_group_create", self.world, C.byref(h))
        self.handle = h
        self._comms: list = []

    def comm(self, rank: int, device: int = 0) -> "LocalComm":
        c = LocalComm(self, rank, device)
        self._comms.append(c)
        return c

    def close(self) -> None:
        from . import _lib

        for c in self._comms:
            c.close()
        self._comms = []
        if getattr(self, "handle", None) is not None and self.handle.value:
            _lib.call("abnn_comm_group_destroy", self.handle)
        self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class LocalComm:
    """Rank ``rank`` of a :class:`LocalGroup`: the ``world`` / ``rank`` of the
    shard layout and the abnn_comm handle ShardedBrain drives (native)."""

    def __init__(self, group: LocalGroup, rank: int, device: int):
        import ctypes as C

        from . import _lib

        self.world, self.rank = group.world, int(rank)
        h = C.c_void_p()
        _lib.call("abnn_comm_create_local", group.handle, self.rank, int(device), C.byref(h))
        self.handle = h

    def close(self) -> None:
        from . import _lib

        if getattr(self, "handle", None) is not None and self.handle.value:
            _lib.call("abnn_comm_destroy", self.handle)
        self.handle = None


class ShardedBrain:
    """The rank-local shard of a graph of ``n_syn_global`` synapses on GPU ``device``.

    native=True (one GPU per rank, RCCL): passes are driven by the C-ABI over
    the library's RCCL communicator (NativeComm, abnn_shard_traverse); False:
    phase by phase from Python around ``comm.all_gather`` (any backend; the
    gloo rehearsal of ranks that share a GPU).  ``comm`` a :class:`LocalComm`:
    the C-driven passes over the in-process group (one thread per rank)."""

    def __init__(self, comm, n_input: int, n_output: int, n_hidden: int, n_syn_global: int,
                 events_per_pass: int, *, device: int = 0, capacity_factor: float = 1.0,
                 native: bool = False, **param_overrides):
        import torch

        self.comm = comm
        self.world, self.rank = comm.world, comm.rank
        lo, hi = shard_ranges(n_syn_global, self.world)[self.rank]
        self.lo, self.hi = lo, hi
        self.n_syn_global = n_syn_global
        self.global_events = global_events(n_syn_global, events_per_pass, self.world,
                                           int(param_overrides.get("mode", 0)))
        cap = int((hi - lo) * capacity_factor) if capacity_factor > 1.0 else 0  # synaptogenesis headroom
        self.brain = Brain(n_input, n_output, n_hidden, hi - lo, events_per_pass, device=device,
                           syn_offset=lo, global_events=self.global_events, syn_capacity=cap,
                           **param_overrides)
        dev = torch.device("cuda", device)
        self._torch = torch
        words = self.brain.exchange_bytes() // 4
        self.xchg = torch.zeros(words, dtype=torch.int32, device=dev)
        self.gathered = torch.zeros(words * self.world, dtype=torch.int32, device=dev)
        self.engine = _GpuEngine(self.brain, lambda: torch.cuda.current_stream(dev))
        self.compact_every = int(self.brain.params.compact_every)
        self._updates = self.brain.structural_updates()
        self.native = None
        if isinstance(comm, LocalComm):
            self.native = comm  # C-driven passes over the in-process group
        elif native:
            # the RCCL communicator spans the same process group as `comm`:
            # rank_offset and the gathered records' order follow its ranks
            self.native = NativeComm(device, group=getattr(comm, "group", None))
            if (self.native.world, self.native.rank) != (self.world, self.rank):
                raise ValueError(f"native communicator is rank {self.native.rank}/{self.native.world}, "
                                 f"the shard layout rank {self.rank}/{self.world}")

    def step(self, passes: int = 1) -> None:
        if self.native is not None:
            from ._lib import call

            call("abnn_shard_traverse", self.brain._h, self.native.handle, int(passes),
                 int(self._torch.cuda.current_stream(self.xchg.device).cuda_stream))
            return
        for _ in range(passes):
            sharded_pass(self.engine, self.comm, self.xchg, self.gathered)
            # every rank runs its structural update after the same pass (the
            # pass index is replicated): re-sum the visited events after one
            if self.compact_every and self.brain.structural_updates() != self._updates:
                self._updates = self.brain.structural_updates()
                self.refresh_global_events()

    def refresh_global_events(self) -> None:
        """A structural update changed every shard's record count, and with it
        the shard's visited events: re-sum them for the clock-tick rule
        (abnn_set_global_events)."""
        t = self._torch.tensor([self.brain.visited_events()], dtype=self._torch.int64, device=self.xchg.device)
        self.comm.all_reduce_sum(t)
        self.global_events = int(t.item())
        self.brain.set_global_events(self.global_events)

    def local_events(self) -> int:
        return self.brain.visited_events()

    def sync_visits(self) -> None:
        """The lazy lastVisited merge (never read by a decision): call on every
        rank before reading or saving lastVisited."""
        if self.native is not None:
            from ._lib import call

            call("abnn_comm_sync_visits", self.brain._h, self.native.handle,
                 int(self._torch.cuda.current_stream(self.xchg.device).cuda_stream))
            return
        merge_visits(self.engine, self.comm)
        self.brain.synchronize()
