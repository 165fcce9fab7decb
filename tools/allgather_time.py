#!/usr/bin/env python3
"""The sharded pass's exchange alone: abnn_shard_traverse's in-place
ncclAllGather of the exchange records (10,272 B per rank at the default
budget) on the library's RCCL communicator, timed by HIP events around
1000 back-to-back calls on one stream, world 1 (the box's one GPU) --
DESIGN.md §7: what the exchange costs before any network."""
import ctypes as C
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist

    from abnn_amd import _lib
    from abnn_amd.shard import NativeComm

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        os.environ.setdefault("MASTER_PORT", str(so.getsockname()[1]))
    dist.init_process_group("gloo", rank=0, world_size=1)
    nc = NativeComm(0)
    lib = _lib.load()
    rec = 10_272
    buf = torch.zeros(rec, dtype=torch.uint8, device="cuda:0")
    f = lib.abnn_debug_comm_allgather
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p]
    f.restype = C.c_int
    for _ in range(50):
        assert f(nc.handle, buf.data_ptr(), rec, 1, None) == 0
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 1000
    a.record()
    assert f(nc.handle, buf.data_ptr(), rec, n, None) == 0
    b.record()
    torch.cuda.synchronize()
    print(f"in-place ncclAllGather of {rec} B per rank, world 1: {a.elapsed_time(b) / n * 1e3:.2f} us per call "
          f"(HIP events around {n} back-to-back calls)")
    nc.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
