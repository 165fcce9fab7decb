"""torchrun worker for tests/test_sharded_gpu.py: every rank runs the product's
ShardedBrain on its shard (GPU), then an unsharded GPU Brain of the whole graph,
and checks its shard, lastFired, clock and rBar against it bit-for-bit."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist

    import abnn_amd
    from abnn_amd.shard import ShardedBrain, TorchComm

    n_syn, events, passes = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    # "native": one GPU per rank, passes driven by the C-ABI over the
    # library's RCCL communicator (abnn_shard_traverse); else ranks share GPU 0
    # and exchange over gloo from Python
    native = len(sys.argv) > 4 and sys.argv[4] == "native"
    dev = int(os.environ.get("LOCAL_RANK", "0")) if native else 0
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl" if native else "gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    # track_visits with a renormalisation after pass 5 (the clock goes back to
    # 0) and a host write of lastVisited ahead of the clock before pass 6, the
    # same on every rank: the lastVisited merge
    extra = dict(track_visits=1, renorm_thresh=4)
    sb = ShardedBrain(TorchComm(), 256, 256, 30_000, n_syn, events, device=dev, native=native, **extra)
    sb.brain.build_random_graph(4)
    sb.brain.set_auto_stimulus(0, 256)

    def at_pass(b, k):
        if k == 6:
            b.set_reward(0.125)
            b.set_last_visited(np.full(8400, b.scalars()["clock"] + 2, np.uint64), 600)

    for k in range(passes):
        at_pass(sb.brain, k)
        sb.step(1)
    torch.cuda.synchronize()
    sb.sync_visits()
    ref = abnn_amd.Brain(256, 256, 30_000, n_syn, events, device=dev, **extra)
    ref.build_random_graph(4)
    ref.set_auto_stimulus(0, 256)
    for k in range(passes):
        at_pass(ref, k)
        ref.encode_traversal(1)
    mine = sb.brain.download_synapses()
    theirs = ref.download_synapses(sb.lo, sb.hi - sb.lo)
    ok = bool(np.array_equal(mine.view(np.uint32), theirs.view(np.uint32)))
    ok &= bool(np.array_equal(sb.brain.last_fired(), ref.last_fired()))
    ok &= bool(np.array_equal(sb.brain.last_visited(), ref.last_visited()))
    ok &= sb.brain.scalars() == ref.scalars()
    ok &= sb.brain.renormalisations() == ref.renormalisations() == 1
    flag = torch.tensor([1 if ok else 0], dtype=torch.int64, device=f"cuda:{dev}" if native else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if sb.native is not None:
        sb.native.close()
    if rank == 0:
        print("SHARDED_OK" if flag.item() == 1 else "SHARDED_MISMATCH", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
