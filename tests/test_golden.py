"""Golden fixtures (tests/golden/*.json, made by tests/golden/make_golden.py).

CPU: the oracle reproduces every fixture (regression pin of the restatement).
GPU: the HIP path reproduces every fixture pass by pass through the C-ABI,
without running the oracle.  Parity against the Metal reference itself is
unpinned."""
import hashlib
import json
import os

import numpy as np
import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = sorted(f[:-5] for f in os.listdir(HERE) if f.endswith(".json"))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8).tobytes()).hexdigest()


def load(name):
    with open(os.path.join(HERE, name + ".json")) as f:
        return json.load(f)


def test_fixtures_present():
    assert {"config1", "c2lite", "renorm_visits"} <= set(CASES)


@pytest.mark.parametrize("name", CASES)
def test_oracle_reproduces_golden(name):
    from oracle import oracle as O

    g = load(name)
    ob = O.OracleBrain(g["n_input"], g["n_output"], g["n_hidden"], g["n_syn"], g["events"],
                       **g["params"])
    ob.build_random_graph(g["seed"], nthreads=8)
    assert sha(ob.syn) == g["initial_synapses_sha256"]
    ob.set_auto_stimulus(*g["stimulus"])
    for rec in g["passes"]:
        if str(rec["pass"]) in g["reward_at"]:
            ob.set_reward(g["reward_at"][str(rec["pass"])])
        ob.pass_serial()
        assert ob.clock == rec["clock"]
        assert int(np.float32(ob.s.rbar).view(np.uint32)) == rec["rbar_bits"]
        assert sha(ob.syn) == rec["synapses_sha256"], rec["pass"]
        assert sha(ob.last_fired) == rec["last_fired_sha256"], rec["pass"]
        st = ob.stats()
        assert {k: st[k] for k in rec["stats"]} == rec["stats"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_gpu_reproduces_golden(gpu, name):
    import abnn_amd

    g = load(name)
    b = abnn_amd.Brain(g["n_input"], g["n_output"], g["n_hidden"], g["n_syn"], g["events"],
                       **g["params"])
    b.build_random_graph(g["seed"])
    assert sha(b.download_synapses()) == g["initial_synapses_sha256"]
    b.set_auto_stimulus(*g["stimulus"])
    for rec in g["passes"]:
        if str(rec["pass"]) in g["reward_at"]:
            b.set_reward(g["reward_at"][str(rec["pass"])])
        b.encode_traversal(1)
        sc = b.scalars()
        assert sc["clock"] == rec["clock"]
        assert int(np.float32(sc["rbar"]).view(np.uint32)) == rec["rbar_bits"]
        assert sha(b.download_synapses()) == rec["synapses_sha256"], rec["pass"]
        assert sha(b.last_fired()) == rec["last_fired_sha256"], rec["pass"]
        if "last_visited_sha256" in rec:
            assert sha(b.last_visited()) == rec["last_visited_sha256"], rec["pass"]
    assert b.stats()["fired"] == g["passes"][-1]["stats"]["fired"]
    syn = b.download_synapses()
    idx = np.array(g["final_sample"]["index"])
    assert syn["w"][idx].view(np.uint32).tolist() == g["final_sample"]["w_bits"]
