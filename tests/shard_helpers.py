"""Test helpers: one sharded pass over `world` shards held in one process,
driven phase by phase around the single exchange (include/abnn/abnn.h):
gate -> all-gather of the records (here: concatenation in rank order) ->
apply -> commit.  What RCCL does across GPUs, done in memory."""
import numpy as np


def oracle_shard_pass(obs) -> None:
    """One pass over oracle shards (OracleBrain list, rank order)."""
    world = len(obs)
    words = obs[0].exchange_words()
    gathered = np.zeros(world * words, dtype=np.int32)
    for r, ob in enumerate(obs):
        ob.shard_gate(gathered[r * words:(r + 1) * words])
    for r, ob in enumerate(obs):
        ob.shard_apply(gathered, world, r)
    for ob in obs:
        ob.shard_commit(gathered, world)


class GpuShards:
    """`world` GPU shard handles on one device with device-resident exchange
    buffers; pass() runs one sharded pass on torch's current stream."""

    def __init__(self, brains, device: int = 0):
        import torch

        self.brains = brains
        self.world = len(brains)
        self.words = brains[0].exchange_bytes() // 4
        dev = torch.device("cuda", device)
        self.gathered = torch.zeros(self.world * self.words, dtype=torch.int32, device=dev)
        self.stream = torch.cuda.current_stream(dev)

    def pass_(self) -> None:
        g, w = self.gathered, self.words
        for r, b in enumerate(self.brains):  # each rank writes its record straight into its slot
            b.shard_gate(g[r * w:(r + 1) * w].data_ptr(), self.stream)
        for r, b in enumerate(self.brains):
            b.shard_apply(g.data_ptr(), self.world, r, self.stream)
        for b in self.brains:
            b.shard_commit(g.data_ptr(), self.world, self.stream)


def merge_visits_local(shards) -> None:
    """The lastVisited merge (abnn.h abnn_shard_visits_delta / _merge) over
    shards held in one process: every shard's deltas, their elementwise MAX
    (what the all-reduce does), the merge on every shard.  Works for oracle
    shards (numpy) and GPU shards (abnn_amd.Brain, torch tensors on the
    current stream)."""
    if hasattr(shards[0], "visits_delta"):  # OracleBrain
        red = np.maximum.reduce([s.visits_delta() for s in shards])
        for s in shards:
            s.visits_merge(red)
        return
    import torch

    dev = torch.device("cuda", shards[0].device)
    stream = torch.cuda.current_stream(dev)
    n = shards[0].n_neuron()
    deltas = [torch.empty(n, dtype=torch.int64, device=dev) for _ in shards]
    for s, d in zip(shards, deltas):
        s.shard_visits_delta(d.data_ptr(), stream)
    red = torch.stack(deltas).amax(dim=0).contiguous()
    for s in shards:
        s.shard_visits_merge(red.data_ptr(), stream)
    stream.synchronize()


def shard_pass_merging(shards, pass_fn) -> None:
    """One sharded pass (pass_fn), then the merge if it renormalised -- the
    rule of abnn_amd.shard.sharded_pass, in one process."""
    before = shards[0].renormalisations()
    pass_fn()
    if shards[0].renormalisations() != before:
        merge_visits_local(shards)
