#!/usr/bin/env python3
"""Rate of the buffer-index launcher (abnn_launch_traversal: the reference's
14-buffer kernel ABI over caller-owned 16-B SynapsePacked records and u32
lastF) at config 3's sweep -- the first 150,000,128 records of the c3 graph,
5,000,512 neurons -- beside the handle API's pass on the same workload.
Prints one JSON line.  usage: python tools/raw_bench.py [passes]"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from abnn_amd import _lib
    from oracle import oracle as O

    passes = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    n_nrn, n_syn, events = 5_000_512, 150_000_128, 150_000_000
    syn = O.gen_synapses(0, n_syn, 256, 256, n_nrn, seed=1, nthreads=16)
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    recs = torch.from_numpy(syn.view(np.uint32).reshape(-1, 4)).to(dev)
    del syn
    lastF = torch.zeros(n_nrn, dtype=torch.int32, device=dev)
    lastV = torch.zeros(n_nrn, dtype=torch.int32, device=dev)
    scal = torch.zeros(4, dtype=torch.int32, device=dev)
    nb = int(lib.abnn_traversal_workspace_bytes(n_syn, events))
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    a = _lib.TraversalArgs()
    p = scal.data_ptr()
    a.syn, a.last_fired, a.last_visited, a.clock = recs.data_ptr(), lastF.data_ptr(), lastV.data_ptr(), p
    a.n_syn, a.tau_vis, a.tau_pre = n_syn, 50_000, 50_000
    a.a_ltp, a.a_ltd, a.w_min, a.w_max = 0.04, 0.02, 0.001, 1.0
    a.budget, a.reward, a.rbar = p + 4, p + 8, p + 12
    a.n_nrn, a.events, a.knobs = n_nrn, events, None
    a.workspace, a.workspace_bytes = ws.data_ptr(), nb

    def one():
        lastF[:256] = scal[0]  # inject_inputs, every input firing (brain.cpp:82)
        scal[1] = 2560         # encode_traversal resets the budget (brain.cpp:90)
        assert lib.abnn_launch_traversal(C.byref(a), None) == 0

    for _ in range(64):  # the start-up transient, as bench.py's settle passes
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(passes):
        one()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / passes
    print(json.dumps({"path": "abnn_launch_traversal (reference layout: 16-B records, u32 lastF)",
                      "workload": "c3 sweep: first 150,000,128 records, 5,000,512 neurons",
                      "passes": passes, "ms_per_pass": round(dt * 1e3, 4),
                      "events_per_s": round(events / dt), "record_bytes_per_s": round(16 * events / dt),
                      "note": "includes the host's two tiny torch writes per pass (inputs, budget)"}), flush=True)


if __name__ == "__main__":
    main()
