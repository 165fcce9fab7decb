"""abnn_amd -- MI355X-native Monte-Carlo synapse traversal engine.

The product is the HIP library ``libabnn_hip.so`` (C-ABI: include/abnn/abnn.h);
this package is its Python host mirror:

* :class:`Brain` -- the reference ``Brain`` (abnn/src/core/brain/brain.h:24-83);
* :mod:`abnn_amd.shard` -- synapse-shard data parallelism over torch.distributed;
* :mod:`abnn_amd.configs` -- the BASELINE.json workloads.
"""
from ._lib import AbnnError, default_params, device_count, load as load_library
from .brain import SYN_DTYPE, Brain, visited_events
from .configs import CONFIGS, Workload

__all__ = [
    "AbnnError", "Brain", "CONFIGS", "SYN_DTYPE", "Workload", "default_params",
    "device_count", "load_library", "visited_events",
]
