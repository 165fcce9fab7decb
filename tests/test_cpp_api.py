"""The C++ Brain API (include/abnn/brain.hpp) end to end: the compiled test
program drives a BrainEngine-style loop on the GPU; the oracle replays it."""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "brain_cpp_test")


def test_cpp_example_builds():
    from abnn_amd.build import build_cpp_example

    assert build_cpp_example() == BIN and os.path.exists(BIN)


@pytest.mark.gpu
def test_cpp_brain_matches_oracle(gpu):
    from abnn_amd.build import build_cpp_example
    from oracle import oracle as O

    build_cpp_example()
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    got = json.loads(r.stdout.strip().splitlines()[-1])

    ob = O.OracleBrain(256, 256, 488, 10_000, 100_000)
    ob.build_random_graph(1)
    v = np.array([0.5 if i % 3 == 0 else 0.0 for i in range(256)], dtype=np.float32)
    fired = 0
    for k in range(24):
        ob.inject_inputs(v, 1000.0)
        if k == 12:
            ob.set_reward(0.5)
        ob.pass_serial()
        fired += int(ob.read_outputs().sum())
    assert got["clock"] == ob.clock
    assert np.float32(got["rbar"]) == np.float32(ob.s.rbar)
    assert got["checksum"] == ob.checksum() == got["copy_checksum"]
    assert got["last_fired_sum"] == int(ob.last_fired.sum())
    assert got["outputs_fired"] == fired
    assert got["mismatch_thrown"] is True

    # the reference caller's code shapes through the buffer views (brain_cpp_test.cpp)
    vb = O.OracleBrain(256, 256, 488, 10_000, 100_000)
    n_nrn = vb.n_neuron()
    i = np.arange(10_000, dtype=np.uint64)
    syn = np.zeros(10_000, dtype=O.SYN_DTYPE)
    syn["src"] = (i * 7919) % n_nrn
    syn["dst"] = (i * 104729 + 13) % n_nrn
    syn["w"] = np.float32(0.1) + (i % 1000).astype(np.float32) / np.float32(1000.0)
    vb.set_synapses(syn)
    budget_sum = outputs = 0
    for k in range(24):
        vb.inject_inputs(v, 1000.0)
        now = vb.clock & 0xFFFFFFFF
        if k % 2 == 0:
            for o in range(256):
                lf = int(vb.last_fired[256 + o]) & 0xFFFFFFFF
                if o % 5 == k % 5 and ((now - lf) & 0xFFFFFFFF) > 1:
                    vb.last_fired[256 + o] = now
        if k == 12:
            vb.set_reward(0.25)
        before = vb.stats()["fired"]
        vb.pass_serial()
        budget_sum += 2560 - (vb.stats()["fired"] - before)
        outputs += int(vb.read_outputs().sum())
    assert got["views_checksum"] == vb.checksum()
    assert got["budget_sum"] == budget_sum
    assert got["views_outputs"] == outputs
    # lastFired and clock both written through their Shared views before one
    # device operation: both writes reached the device (brain.hpp)
    assert got["shared_both_ok"] is True
