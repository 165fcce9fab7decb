#!/usr/bin/env python3
"""Generate tests/golden/*.json from the C oracle (serial C1 loop).

PARITY UNPINNED against the reference itself: tjamescouch/abnn ships no tests,
fixtures or golden vectors, and brain.metal cannot be built or run in this
image.  These files pin the oracle (regression) and give the
GPU path a fixed target that does not need the oracle at run time.  Each
fixture records, per pass: SHA-256 of the synapse array and of lastFired,
clock, rBar bits and the pass statistics, plus a sparse sample of records.

    python tests/golden/make_golden.py        # rewrites the fixtures
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

CASES = {
    # BASELINE configs[0]: 1k neurons, 10k synapses, 100k events (all input->output)
    "config1": dict(n_hidden=488, n_syn=10_000, events=100_000, passes=64, seed=1,
                    reward_at={20: 1.0, 40: -0.5}, params={}),
    # "C-2-lite" of SURVEY §4: 100k neurons, 1M synapses: all-gated passes 3-5,
    # then the budget-saturated steady state
    "c2lite": dict(n_hidden=99_488, n_syn=1_000_000, events=1_000_000, passes=12, seed=1,
                   reward_at={8: 0.25}, params={}),
    # renormalisation + lastVisited tracking + a small budget
    "renorm_visits": dict(n_hidden=20_000, n_syn=200_000, events=150_000, passes=16, seed=3,
                          reward_at={5: 0.5}, params=dict(renorm_thresh=6, track_visits=1,
                                                           max_spikes=300)),
}


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8).tobytes()).hexdigest()


def run_case(name, c):
    from oracle import oracle as O

    ob = O.OracleBrain(256, 256, c["n_hidden"], c["n_syn"], c["events"], **c["params"])
    ob.build_random_graph(c["seed"], nthreads=8)
    ob.set_auto_stimulus(0, 256)
    sample_idx = np.unique(np.linspace(0, c["n_syn"] - 1, 97).astype(np.int64))
    out = {"name": name, "n_input": 256, "n_output": 256, "n_hidden": c["n_hidden"],
           "n_syn": c["n_syn"], "events": c["events"], "seed": c["seed"],
           "params": c["params"], "reward_at": {str(k): v for k, v in c["reward_at"].items()},
           "stimulus": [0, 256], "initial_synapses_sha256": sha(ob.syn), "passes": []}
    for k in range(c["passes"]):
        if k in c["reward_at"]:
            ob.set_reward(c["reward_at"][k])
        ob.pass_serial()
        rec = {"pass": k, "clock": ob.clock,
               "rbar_bits": int(np.float32(ob.s.rbar).view(np.uint32)),
               "synapses_sha256": sha(ob.syn), "last_fired_sha256": sha(ob.last_fired),
               "stats": ob.stats()}
        if c["params"].get("track_visits"):
            rec["last_visited_sha256"] = sha(ob.last_visited)
        out["passes"].append(rec)
    out["final_sample"] = {"index": sample_idx.tolist(),
                           "w_bits": ob.syn["w"][sample_idx].view(np.uint32).tolist()}
    out["final_last_fired_head"] = ob.last_fired[:1024].tolist()
    return out


def main():
    from abnn_amd.build import build_oracle

    build_oracle()
    for name, c in CASES.items():
        data = run_case(name, c)
        with open(os.path.join(HERE, f"{name}.json"), "w") as f:
            json.dump(data, f, indent=1)
        print("wrote", name, len(data["passes"]), "passes")


if __name__ == "__main__":
    main()
