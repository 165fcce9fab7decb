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
