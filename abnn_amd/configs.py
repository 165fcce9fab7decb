"""The workloads of BASELINE.json ``configs``.

N_NRN = n_input + n_output + n_hidden (brain.cpp:24); n_input = n_output = 256
(constants.h:2-3).  ``events`` is EVENTS_PER_PASS; the visited events per pass are
min(roundup(events,256), n_syn).
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class Workload:
    name: str
    n_input: int
    n_output: int
    n_hidden: int
    n_syn: int
    events: int
    note: str

    @property
    def n_neuron(self) -> int:
        return self.n_input + self.n_output + self.n_hidden


CONFIGS = {
    # configs[0]: CPU plumbing case, golden fixtures
    "c1": Workload("c1", 256, 256, 1000 - 512, 10_000, 100_000,
                   "N_NRN=1k, N_SYN=10k, EVENTS=100k (10k visits/pass)"),
    # configs[1]: kernel bring-up and full-state parity
    "c2": Workload("c2", 256, 256, 100_000 - 512, 10_000_000, 10_000_000,
                   "N_NRN=100k, N_SYN=10M, 10M events/pass"),
    # configs[2]: constants.h defaults -- the headline single-GPU workload
    "c3": Workload("c3", 256, 256, 5_000_000, 1_000_000_000, 150_000_000,
                   "N_NRN=5,000,512, N_SYN=1B (16 GB as SynapsePacked; 11 GB as the packed src/dst/w streams in HBM), 150M events/pass"),
    # configs[3]: the same graph sharded across GPUs (150M events/pass/GPU, capped by shard)
    "c4": Workload("c4", 256, 256, 5_000_000, 1_000_000_000, 150_000_000,
                   "N_NRN=5,000,512, N_SYN=1B split into one contiguous shard per GPU, 150M events/pass/GPU"),
    # configs[4]: HBM-filling graph (64 GB as SynapsePacked, 44 GB packed; 5.5 GB per GPU at 8 ways).
    # One GPU holds it whole (bench.py --config c5 runs it there); the label
    # follows the shard count the run actually uses (bench.py workload_label)
    "c5": Workload("c5", 256, 256, 5_000_000, 4_000_000_000, 150_000_000,
                   "N_NRN=5,000,512, N_SYN=4B (HBM-filling), 150M events/pass/GPU"),
}
