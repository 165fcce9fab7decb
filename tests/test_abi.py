"""CPU checks of the drop-in boundary: the HIP library loads, exports every
symbol include/abnn/abnn.h declares, the ctypes mirrors match the C layouts,
and the no-GPU path fails loudly instead of falling back."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "abnn", "abnn.h")
DEBUG_HEADER = os.path.join(ROOT, "include", "abnn", "abnn_debug.h")


def declared_functions(header=HEADER):
    src = open(header).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\*?\s*(abnn_[a-z0-9_]+)\s*\(",
                                 src, flags=re.M)))


def test_library_exports_every_declared_symbol():
    from abnn_amd import _lib

    lib = C.CDLL(_lib.LIB_PATH)
    names = declared_functions()
    assert len(names) >= 35
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert set(names) == bound, set(names) ^ bound


def test_exported_symbols_are_exactly_the_declared_ones():
    """Every abnn_* function the library exports is declared in abnn.h (the
    boundary) or abnn_debug.h (diagnostics, outside the stable ABI)."""
    from abnn_amd import _lib

    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if re.search(r" T abnn_", ln)}
    declared = set(declared_functions()) | set(declared_functions(DEBUG_HEADER))
    assert exported == declared, exported ^ declared
    assert not set(declared_functions()) & set(declared_functions(DEBUG_HEADER))


def test_struct_layouts_match_c(tmp_path):
    from abnn_amd import _lib
    from oracle import oracle as O

    prog = tmp_path / "sz.c"
    prog.write_text('#include "abnn/abnn.h"\n#include <stdio.h>\n#include <stddef.h>\n'
                    'int main(void){printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(abnn_synapse),'
                    'sizeof(abnn_dims), sizeof(abnn_params), sizeof(abnn_scalars), sizeof(abnn_stats),'
                    'sizeof(abnn_state), offsetof(abnn_params, renorm_thresh), sizeof(abnn_layout),'
                    'sizeof(abnn_traversal_args), offsetof(abnn_traversal_args, workspace));return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(prog)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    want = [16, C.sizeof(_lib.Dims), C.sizeof(_lib.Params), C.sizeof(_lib.Scalars),
            C.sizeof(_lib.Stats), C.sizeof(_lib.State), _lib.Params.renorm_thresh.offset,
            C.sizeof(_lib.Layout), C.sizeof(_lib.TraversalArgs), _lib.TraversalArgs.workspace.offset]
    assert got == want
    assert C.sizeof(O.Params) == C.sizeof(_lib.Params) and C.sizeof(O.Dims) == C.sizeof(_lib.Dims)


def test_default_params_equal_oracle():
    from abnn_amd import _lib
    from oracle import oracle as O

    a, b = _lib.default_params(), O.default_params()
    for name, _ in _lib.Params._fields_:
        assert getattr(a, name) == getattr(b, name), name


def test_abi_version_and_status_strings():
    from abnn_amd import _lib

    lib = _lib.load()
    assert lib.abnn_abi_version() == _lib.ABI_VERSION == 10
    assert lib.abnn_status_string(0) == b"ok"
    assert lib.abnn_status_string(4) == b"size mismatch"


def test_no_gpu_fails_loudly():
    import abnn_amd

    if abnn_amd.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(abnn_amd.AbnnError) as e:
        abnn_amd.Brain(256, 256, 488, 10_000, 100_000)
    assert e.value.status == 6  # ABNN_ERR_NO_DEVICE


def test_missing_library_is_an_import_error(monkeypatch, tmp_path):
    from abnn_amd import _lib

    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(ImportError):
        _lib.load()


def test_gpu_kernels_built_for_gfx950():
    from abnn_amd import _lib

    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    assert b"k_gate" in data


def test_shard_partition_helpers():
    from abnn_amd.shard import global_events, shard_ranges

    r = shard_ranges(10, 3)
    assert r == [(0, 4), (4, 7), (7, 10)]
    assert shard_ranges(1_000_000_000, 8)[7] == (875_000_000, 1_000_000_000)
    assert global_events(1_000_000_000, 150_000_000, 1) == 150_000_128
    assert global_events(1_000_000_000, 150_000_000, 8) == 1_000_000_000
    assert global_events(1_000_000_000, 150_000_000, 2) == 2 * 150_000_128


def _src_code(n):
    """abnn.h (abnn_state): the filter code of a 24-bit src, as (lo, hi)."""
    n = n.astype(np.uint64)
    b, j = n & 31, (n >> 5) & 0x7FFFF
    jh = j >> 13
    t = jh * 0x9E5
    g, hb = (j ^ t) & 8191, (b + t) & 31
    return (g << 3 | (hb & 7)), (b | (jh >> 5) << 5 | (hb >> 3) << 6)


def _code_src(lo, hi):
    g, b = lo >> 3, hi & 31
    hb = (lo & 7) | (hi >> 6) << 3
    jh = (((hb - b) * 13) & 31) | ((hi >> 5) & 1) << 5
    j = ((g ^ jh * 0x9E5) & 8191) | jh << 13
    return j << 5 | b


def test_src_code_is_a_bijection_matching_the_filter():
    """The stored src layout (layout 3): every 24-bit src has a distinct
    (lo, hi), the documented inverse restores it, lo >> 3 is the src's filter
    block, hi & 31 its low bit and lo & 7 | hi >> 6 << 3 its high bit (the
    word hash filter_t / filter_set of kernels.hip)."""
    n = np.arange(1 << 24, dtype=np.uint64)
    lo, hi = _src_code(n)
    assert lo.max() < 1 << 16 and hi.max() < 1 << 8
    assert np.unique(lo | hi << 16).size == 1 << 24
    assert np.array_equal(_code_src(lo, hi), n)
    j, b = n >> 5, n & 31
    t = (j >> 13) * 0x9E5
    assert np.array_equal(lo >> 3, (j ^ t) & 8191)
    assert np.array_equal(hi & 31, b)
    assert np.array_equal((lo & 7) | (hi >> 6) << 3, (b + t) & 31)


def _raw_ws_bytes(n_syn: int, events: int) -> tuple[int, int]:
    """raw.hip's workspace: header, filter (8192 x 8 B), per 1024-event group
    {candidates, prefix, survivors + sequence start}, per 4096 groups a scan
    total, per gate wave (4096) its
    stored limit, statistics and chunk table, the spike list (min(E, 65536)) -- and the
    recommended pool of 4-KiB survivor chunks: one per wave + E/64 entries + 64.
    The fused pass adds a look-back word per gate workgroup (256), three sets of
    257 workgroup range bounds, two of 256 range costs and 8 u64 per gate wave
    of diagnostics."""
    al = lambda x: (x + 15) & ~15
    E = min((events + 255) // 256 * 256, n_syn)
    g, W = (E + 1023) // 1024, 4096
    maxc = (g + W - 1) // W * 4 + 1
    fixed = 128 + 8192 * 8 + 2 * al(4 * g) + al(4 * ((g + 4095) // 4096)) + al(16 * g) + al(4 * W) + al(8 * W) + \
        al(4 * W * maxc) + al(4 * min(E, 65536)) + 8 * 256 + al(4 * 3 * 257) + 4 * 2 * 256 + 8 * 8 * W
    pool = (W + (E // 64 + 255) // 256 + 64) * 4096 if E else 0
    return fixed, fixed + pool


def test_workspace_bytes_of_the_buffer_index_launcher():
    """abnn_traversal_workspace_bytes / _min_bytes: a bounded survivor pool
    (~60 MB at config 3, was 16 B per visited event = 2.4 GB) over fixed
    per-group and per-wave counters."""
    from abnn_amd import _lib

    lib = _lib.load()
    for n_syn, ev in ((0, 100), (10_000, 100_000), (150_000_128, 150_000_000), (1_000_000_000, 150_000_000),
                      (3_000, 4_097), (4_000_000_000, 4_000_000_000)):
        fixed, rec = _raw_ws_bytes(n_syn, ev)
        assert lib.abnn_traversal_workspace_min_bytes(n_syn, ev) == fixed, (n_syn, ev)
        assert lib.abnn_traversal_workspace_bytes(n_syn, ev) == rec, (n_syn, ev)
    ws = lib.abnn_traversal_workspace_bytes
    assert ws(1_000_000_000, 150_000_000) == ws(150_000_128, 150_000_000)  # only visited events
    assert ws(1_000_000_000, 150_000_000) < 70_000_000  # bounded: < 0.5 B per visited event


def test_launcher_rejects_bad_arguments():
    from abnn_amd import _lib

    lib = _lib.load()
    a = _lib.TraversalArgs()
    assert lib.abnn_launch_traversal(C.byref(a), None) == 1  # ABNN_ERR_INVALID: null buffers
