"""ctypes binding of the C-ABI in include/abnn/abnn.h (libabnn_hip.so).

The library is built in-tree by ``abnn_amd.build.build_hip()`` (hipcc,
--offload-arch=gfx950).  There is no fallback: if the shared object is missing
or does not export the ABI, importing the product fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# ABNN_LIB: another build of the same ABI (A/B timing of kernel variants,
# tools/ab_variants.sh); the default is the in-tree product library
LIB_PATH = os.environ.get("ABNN_LIB") or os.path.join(_HERE, "libabnn_hip.so")

SUMMARY_WORDS = 4
COMM_ID_BYTES = 128


class Dims(C.Structure):
    """abnn_dims -- Brain(nInput, nOutput, nHidden, nSynapses, eventsPerPass), brain.h:27-31."""

    _fields_ = [
        ("n_input", C.c_uint32),
        ("n_output", C.c_uint32),
        ("n_hidden", C.c_uint64),
        ("n_syn", C.c_uint64),
        ("events_per_pass", C.c_uint64),
        ("syn_offset", C.c_uint64),
        ("global_events", C.c_uint64),
        ("syn_capacity", C.c_uint64),
    ]


class Params(C.Structure):
    """abnn_params -- every knob of brain.metal:22-31, constants.h:16-19, brain.h:17-19."""

    _fields_ = [
        ("base_scale", C.c_float),
        ("refractory", C.c_uint32),
        ("window_pre", C.c_uint32),
        ("clock_inc", C.c_uint32),
        ("target_rate_hz", C.c_float),
        ("eta_home", C.c_float),
        ("eta_reward", C.c_float),
        ("alpha_rbar", C.c_float),
        ("a_ltp", C.c_float),
        ("a_ltd", C.c_float),
        ("w_min", C.c_float),
        ("w_max", C.c_float),
        ("max_spikes", C.c_uint32),
        ("tick_ns", C.c_uint32),
        ("tau_vis", C.c_uint32),
        ("tau_pre", C.c_uint32),
        ("renorm_thresh", C.c_uint64),
        ("track_visits", C.c_uint32),
        ("mode", C.c_uint32),
        ("seed", C.c_uint64),
        ("w_prune", C.c_float),
        ("p_new", C.c_float),
        ("w_init", C.c_float),
        ("compact_every", C.c_uint32),
    ]


class Scalars(C.Structure):
    _fields_ = [("clock", C.c_uint64), ("reward", C.c_float), ("rbar", C.c_float),
                ("pass_index", C.c_uint64)]


MODE_SWEEP, MODE_RANDOM = 0, 1  # abnn_params.mode (include/abnn/abnn.h)
ABI_VERSION = 10
LAYOUT_VERSION = 4


class Stats(C.Structure):
    _fields_ = [
        ("passes", C.c_uint64),
        ("events", C.c_uint64),
        ("pre_gated", C.c_uint64),
        ("post_gated", C.c_uint64),
        ("updated", C.c_uint64),
        ("fired", C.c_uint64),
        ("pruned", C.c_uint64),
        ("grown", C.c_uint64),
    ]

    def as_dict(self) -> dict:
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


class State(C.Structure):
    _fields_ = [
        ("synapses", C.c_void_p),  # opaque device records (abnn_synapse_layout)
        ("last_fired", C.c_void_p),
        ("last_visited", C.c_void_p),
        ("clock", C.c_void_p),
        ("reward", C.c_void_p),
        ("rbar", C.c_void_p),
    ]


LAYOUT_MAX_ARRAYS = 4


class ArrayDesc(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("bytes", C.c_uint64), ("elem_bytes", C.c_uint32), ("name", C.c_char * 20)]


class Layout(C.Structure):
    """abnn_layout -- the device record layout behind abnn_state.synapses (versioned apart from the ABI)."""

    _fields_ = [("version", C.c_uint32), ("n_arrays", C.c_uint32), ("arrays", ArrayDesc * LAYOUT_MAX_ARRAYS)]


class TraversalArgs(C.Structure):
    """abnn_traversal_args -- monte_carlo_traversal's 14 buffers (brain.metal:42-58), caller-owned."""

    _fields_ = [
        ("syn", C.c_void_p), ("last_fired", C.c_void_p), ("last_visited", C.c_void_p), ("clock", C.c_void_p),
        ("n_syn", C.c_uint32), ("tau_vis", C.c_uint32), ("tau_pre", C.c_uint32),
        ("a_ltp", C.c_float), ("a_ltd", C.c_float), ("w_min", C.c_float), ("w_max", C.c_float),
        ("budget", C.c_void_p), ("reward", C.c_void_p), ("rbar", C.c_void_p),
        ("n_nrn", C.c_uint32), ("events", C.c_uint32), ("knobs", C.c_void_p),
        ("workspace", C.c_void_p), ("workspace_bytes", C.c_uint64),
    ]


class AbnnError(RuntimeError):
    def __init__(self, fn: str, status: int, msg: str):
        super().__init__(f"{fn} failed: status {status} ({msg})")
        self.status = status


# Every symbol include/abnn/abnn.h declares: (name, restype, argtypes).
_VP, _U32, _U64, _I32, _F = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int, C.c_float
_PU64, _PU32 = C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)
SIGNATURES = [
    ("abnn_abi_version", C.c_int, []),
    ("abnn_status_string", C.c_char_p, [C.c_int]),
    ("abnn_last_error", C.c_char_p, []),
    ("abnn_default_params", None, [C.POINTER(Params)]),
    ("abnn_device_count", C.c_int, []),
    ("abnn_brain_create", C.c_int, [C.POINTER(Dims), C.POINTER(Params), C.c_int, C.POINTER(_VP)]),
    ("abnn_brain_destroy", C.c_int, [_VP]),
    ("abnn_get_dims", C.c_int, [_VP, C.POINTER(Dims)]),
    ("abnn_get_params", C.c_int, [_VP, C.POINTER(Params)]),
    ("abnn_state_ptrs", C.c_int, [_VP, C.POINTER(State)]),
    ("abnn_synapse_layout", C.c_int, [_VP, C.POINTER(Layout)]),
    ("abnn_n_neuron", C.c_uint64, [_VP]),
    ("abnn_upload_synapses", C.c_int, [_VP, _U64, _VP, _U64]),
    ("abnn_download_synapses", C.c_int, [_VP, _U64, _VP, _U64]),
    ("abnn_generate_synapses", C.c_int, [_VP, _U64]),
    ("abnn_checksum_synapses", C.c_int, [_VP, _PU64]),
    ("abnn_get_last_fired", C.c_int, [_VP, _U64, _VP, _U64]),
    ("abnn_set_last_fired", C.c_int, [_VP, _U64, _VP, _U64]),
    ("abnn_get_last_visited", C.c_int, [_VP, _U64, _VP, _U64]),
    ("abnn_set_last_visited", C.c_int, [_VP, _U64, _VP, _U64]),
    ("abnn_set_timestamps", C.c_int, [_VP, _VP, _U64, _U64]),
    ("abnn_get_scalars", C.c_int, [_VP, C.POINTER(Scalars)]),
    ("abnn_set_scalars", C.c_int, [_VP, C.POINTER(Scalars)]),
    ("abnn_set_reward", C.c_int, [_VP, _F]),
    ("abnn_inject_inputs", C.c_int, [_VP, _VP, _U32, _F]),
    ("abnn_read_outputs", C.c_int, [_VP, _VP, _U32]),
    ("abnn_set_auto_stimulus", C.c_int, [_VP, _U64, _U64]),
    ("abnn_traverse", C.c_int, [_VP, _U32, _VP]),
    ("abnn_synchronize", C.c_int, [_VP, _VP]),
    ("abnn_exchange_bytes", C.c_uint64, [_VP]),
    ("abnn_set_global_events", C.c_int, [_VP, _U64]),
    ("abnn_shard_gate", C.c_int, [_VP, _VP, _VP]),
    ("abnn_shard_apply", C.c_int, [_VP, _VP, _U32, _U32, _VP]),
    ("abnn_shard_commit", C.c_int, [_VP, _VP, _U32, _VP]),
    ("abnn_get_budget", C.c_int, [_VP, _PU32]),
    ("abnn_structural_updates", C.c_uint64, [_VP]),
    ("abnn_shard_visits_delta", C.c_int, [_VP, _VP, _VP]),
    ("abnn_shard_visits_merge", C.c_int, [_VP, _VP, _VP]),
    ("abnn_renormalisations", C.c_uint64, [_VP]),
    ("abnn_traversal_workspace_bytes", C.c_uint64, [_U32, _U32]),
    ("abnn_traversal_workspace_min_bytes", C.c_uint64, [_U32, _U32]),
    ("abnn_traversal_workspace_error", C.c_int, [_VP, _PU32, _VP]),
    ("abnn_launch_traversal", C.c_int, [C.POINTER(TraversalArgs), _VP]),
    ("abnn_launch_renormalise", C.c_int, [_VP, _VP, _VP, _U32, _VP]),
    ("abnn_comm_unique_id", C.c_int, [_VP]),
    ("abnn_comm_create", C.c_int, [_VP, _U32, _U32, C.c_int, C.POINTER(_VP)]),
    ("abnn_comm_destroy", C.c_int, [_VP]),
    ("abnn_shard_traverse", C.c_int, [_VP, _VP, _U32, _VP]),
    ("abnn_comm_sync_visits", C.c_int, [_VP, _VP, _VP]),
    ("abnn_comm_group_create", C.c_int, [_U32, C.POINTER(_VP)]),
    ("abnn_comm_group_destroy", C.c_int, [_VP]),
    ("abnn_comm_create_local", C.c_int, [_VP, _U32, C.c_int, C.POINTER(_VP)]),
    ("abnn_get_stats", C.c_int, [_VP, C.POINTER(Stats)]),
    ("abnn_reset_stats", C.c_int, [_VP]),
    ("abnn_enable_timing", C.c_int, [_VP, C.c_int]),
    ("abnn_get_kernel_time", C.c_int, [_VP, C.POINTER(C.c_double), _PU64]),
    ("abnn_get_kernel_times", C.c_int, [_VP, _VP, _U64, _PU64]),
    ("abnn_save_bnn", C.c_int, [_VP, C.c_char_p]),
    ("abnn_load_bnn", C.c_int, [_VP, C.c_char_p]),
    ("abnn_save_flat", C.c_int, [_VP, C.c_char_p]),
    ("abnn_load_flat", C.c_int, [_VP, C.c_char_p]),
]

# entry points new in ABI 10: an older A/B variant build (ABNN_LIB, timing only) may lack them
ABI10_ADDITIONS = ("abnn_comm_group_create", "abnn_comm_group_destroy", "abnn_comm_create_local")

_lib = None


def _share_hip_runtime_with_torch() -> None:
    """PyTorch-ROCm wheels bundle their own libamdhip64/libhsa-runtime64.  If
    this library pulled in /opt/rocm's copy first, a later `import torch` would
    load a second HIP runtime into the process and fail to see the GPU.  When
    torch is installed, preload its runtime (by path, without importing torch)
    so both resolve libamdhip64.so.7 to the same object whatever the import
    order; without torch the system ROCm runtime is used."""
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    hip = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
    if os.path.exists(hip):
        C.CDLL(hip, mode=C.RTLD_GLOBAL)


# diagnostics (include/abnn/abnn_debug.h, outside the stable boundary)
DEBUG_SIGNATURES = [
    ("abnn_debug_set_wave_clock", C.c_int, [_VP, C.c_int]),
    ("abnn_debug_raw_stats", C.c_int, [_VP, C.POINTER(C.c_uint64), _VP]),
    ("abnn_debug_raw_gate_timing", C.c_int, [C.c_int]),
    ("abnn_debug_raw_gate_time", C.c_int, [C.POINTER(C.c_double), _PU32]),
    ("abnn_debug_raw_fused", C.c_int, [C.c_int]),
    ("abnn_debug_raw_fused_active", C.c_int, []),
    ("abnn_debug_raw_wave_clock", C.c_int, [_VP, C.c_uint64, _U32, _U32, C.POINTER(C.c_uint64), C.c_uint64, _VP]),
]


def load() -> C.CDLL:
    """Load libabnn_hip.so (built in-tree); raise if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback for the traversal engine)")
    _share_hip_runtime_with_torch()
    lib = C.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES + DEBUG_SIGNATURES:
        if not hasattr(lib, name) and ((name, res, args) in DEBUG_SIGNATURES or
                                       (os.environ.get("ABNN_LIB") and name in ABI10_ADDITIONS)):
            continue  # an older variant build (A/B timing) without this diagnostic / entry point
        fn = getattr(lib, name)  # AttributeError = the ABI is not exported
        fn.restype = res
        fn.argtypes = args
    got = lib.abnn_abi_version()
    if got != ABI_VERSION:
        # an A/B timing build of another ABI version only with an explicit
        # opt-in: its state layout and record encoding may differ
        if not os.environ.get("ABNN_LIB_ANY_ABI"):
            raise ImportError(f"{LIB_PATH}: ABI version {got}, this binding is {ABI_VERSION} "
                              "(ABNN_LIB_ANY_ABI=1 accepts it for pass timing only)")
        import warnings

        warnings.warn(f"{LIB_PATH}: ABI version {got} != {ABI_VERSION}; use pass/timing entry points only")
    _lib = lib
    return lib


def check(fn_name: str, status: int) -> None:
    if status != 0:
        lib = load()
        msg = lib.abnn_last_error().decode(errors="replace")
        raise AbnnError(fn_name, status, msg)


def call(fn_name: str, *args) -> None:
    lib = load()
    check(fn_name, getattr(lib, fn_name)(*args))


def default_params(**overrides) -> Params:
    p = Params()
    load().abnn_default_params(C.byref(p))
    for k, v in overrides.items():
        if not hasattr(p, k):
            raise KeyError(k)
        setattr(p, k, v)
    return p


def device_count() -> int:
    return int(load().abnn_device_count())
