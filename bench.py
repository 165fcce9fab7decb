#!/usr/bin/env python3
"""Benchmark: traversal events/s of the C1 synapse sweep on MI355X.

Workload (BASELINE.json configs[2], constants.h defaults): N_NRN = 5,000,512
(256 in + 256 out + 5M hidden), N_SYN = 1e9 (12 GB of src/dst/w arrays in
HBM; SynapsePacked's never-read pad is not stored), EVENTS_PER_PASS = 150M
(150,000,128 visits per pass).  Synthetic graph =
the build_random_graph recipe (brain-engine.cpp:31-53) with the portable RNG,
generated on the GPU; every pass stamps all 256 inputs.

One "step" = one whole pass: stimulus + bitmap + streaming gate + budget scan +
apply + finalize (+ the two exchanges at N>1).  `value` = visited events of all
ranks per second over the K timed steps (max over ranks of the wall time).
Before the W warm-up passes, --settle untimed passes (default 64) take the
freshly built graph through its start-up transient (lastFired = 0 gates every
event in passes 0-5); the JSON reports them (config.settle_passes/settle_s).

N > 1 (torchrun, one process per GPU, RCCL): the 1B-synapse graph is split in
N contiguous shards; every GPU sweeps 150M events of its shard per pass
(capped by the shard: 125M at N = 8), so per-GPU work is fixed -> "weak".

Extra JSON fields: `roofline` (the gate kernel: algorithmic bytes per launch /
its HIP-event-timed average duration vs 8 TB/s) and `cpu_baseline` (the
threaded C oracle on this host, rank 0 at N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# Start-up transient of a freshly built brain: lastFired = 0
# makes passes 0-5 gate every event (passes 3-5 run the refractory stage on all
# 150M), passes 6-9 drain it, and the recent set grows from ~8k to ~13k
# neurons over passes ~42-55 as the spikes leave the 256 outputs.  These
# passes run before warm-up, untimed, like loading a running brain.
SETTLE_PASSES = 64


def timing_every(steps: int) -> int:
    """Gate launches sampled by HIP events (the roofline's average duration):
    every 4th in short runs, every 8th from 100 timed passes on."""
    return 4 if steps < 100 else 8


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200,
                    help="timed passes (the reference engine runs passes forever; 200 x ~0.13 ms)")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--settle", type=int, default=SETTLE_PASSES,
                    help="untimed passes from the freshly built graph to the steady state, before "
                         "the warm-up (the start-up transient, DESIGN.md §6)")
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c5"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the CPU baseline (0: every CPU this process may run on)")
    ap.add_argument("--cpu-passes", type=int, default=3)
    ap.add_argument("--mode", choices=["sweep", "random"], default="sweep",
                    help="sweep: event t visits synapse t (the reference kernel); random: "
                         "README §4 random-edge picks (include/abnn/abnn.h)")
    ap.add_argument("--events", type=int, default=0,
                    help="override EVENTS_PER_PASS (e.g. = N_SYN for the config-3 full sweep)")
    ap.add_argument("--shard-path", action="store_true",
                    help="at one GPU, run the sharded pass (abnn_shard_traverse over the library's RCCL "
                         "communicator, world 1) instead of the fused single-GPU pass: its per-pass "
                         "overhead (DESIGN.md §7)")
    ap.add_argument("--no-reference-layout", action="store_true",
                    help="skip the reference_layout sub-object of the default run")
    ap.add_argument("--raw", action="store_true",
                    help="the reference-layout path: abnn_launch_traversal (brain.metal's 14-buffer ABI) over "
                         "caller-owned 16-B SynapsePacked records and u32 lastF at the config's sweep "
                         "(DESIGN.md §5, include/abnn/abnn.h)")
    ap.add_argument("--plasticity", action="store_true",
                    help="config-5 dynamics: reward-modulated STDP (reward 0.25) with pruning "
                         "(w < 0.105) and synaptogenesis (p_new 0.25, w_init 0.5, +1%% capacity), "
                         "structural update every 50 passes (README §5, include/abnn/abnn.h)")
    return ap.parse_args()


PLASTICITY = dict(w_prune=0.105, p_new=0.25, w_init=0.5, compact_every=50)


def algorithmic_bytes(stats: dict, track_visits: bool, random_mode: bool = False) -> int:
    """Bytes the streaming gate kernel must move from HBM: the
    3-B (24-bit) src of every visited event -- the records are held as arrays
    and the pre-spike gate reads nothing else (+4 B dst read and 8 B
    lastVisited write per event with track_visits).  The pre-spike lookup of
    lastFired[src] is served by the per-pass LDS filter / L2 bitmap, built by
    the pass from the last passes' spike lists (k_bitmap, after host writes,
    reads lastFired once: 8 B per neuron).  Random mode: every pick is one
    random access to the 4-GB src32 mirror, and HBM moves a whole 64-B line
    for it: 64 B per pick (the 4 useful bytes are 1/16 of that)."""
    e = stats["events"]
    return (64 if random_mode else 3) * e + (12 * e if track_visits else 0)


def survey_bytes(stats: dict, track_visits: bool) -> int:
    """SURVEY.md §8(d) per-event figure for the same work: 24 B per visited event
    (16 B record + 8 B lastFired[src]) + 8 B lastFired[dst] per pre-gated event."""
    e = stats["events"]
    return 24 * e + (8 * e if track_visits else 0) + 8 * stats["pre_gated"]


def load_traffic(config: str):
    """The committed PMC traffic record (tools/profile.sh -> tools/pmc_summary.py)
    if it was measured on these kernel sources; else (None, why)."""
    from abnn_amd.build import kernel_source_sha

    p = os.path.join(ROOT, "profiles", f"traffic_{config}.json")
    if not os.path.exists(p):
        return None, "no profiles/traffic_%s.json" % config
    try:
        with open(p) as f:
            t = json.load(f)
    except (OSError, ValueError) as e:
        return None, f"unreadable traffic record: {e}"
    sha = kernel_source_sha()
    if t.get("source_sha") != sha:
        return None, (f"stale: traffic_{config}.json was measured on kernel sources {t.get('source_sha')}, "
                      f"this tree is {sha} (re-run tools/profile.sh)")
    return t, None


def host_cpus() -> dict:
    """The CPUs the CPU baseline may use: the affinity set (what a thread pool
    can be scheduled on), the machine's count, and the cgroup CPU quota when
    one is set (a quota below the affinity set caps the threads' real rate)."""
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"available": avail, "machine": os.cpu_count(), "cgroup_quota_cpus": quota}


def cpu_baseline(wl, events: int, mode: int, threads: int, timed_passes: int, extra: dict,
                 settle: int) -> dict:
    """The threaded C oracle ("port") on the host cores.  Sweep: the pass only
    ever touches the first E synapses, so the sample holds exactly those and
    produces the identical pass results (same settle passes as the GPU run, so
    the same steady state).  Random mode: picks span the whole graph, so the
    sample is a graph of at most 150M synapses (bounded host memory and
    generation time) with the same neurons and events -- a REDUCED graph: the
    picks hit a smaller working set than the GPU's, which likely overstates
    the CPU rate."""
    from oracle import oracle as O

    reduced = False
    if mode == 1:
        n_syn = min(wl.n_syn, 150_000_000)
        reduced = n_syn < wl.n_syn
        E = O.visited_events(events, n_syn, 1)
        what = f"{n_syn:,}-synapse random graph ({wl.name} recipe), {E:,} random picks per pass"
    else:
        n_syn = E = O.visited_events(events, wl.n_syn)
        what = f"first {E:,} synapses of the {wl.name} graph (all the sweep touches)"
    ob = O.OracleBrain(wl.n_input, wl.n_output, wl.n_hidden, n_syn, events, mode=mode,
                       syn_capacity=int(n_syn * 1.01) if extra else 0, **extra)
    ob.build_random_graph(1, nthreads=threads)
    ob.set_auto_stimulus(0, wl.n_input)
    if extra:
        ob.set_reward(0.25)
        what += " with the same plasticity settings"
    ob.pass_threaded(settle, nthreads=min(threads, 64))
    # timed passes at 16, 64 and every available thread (the oracle caps a
    # pass at 256): the box's cgroup CPU quota can make fewer threads faster
    # (profiles/r04b_cpu_thread_scaling.txt); the best is the baseline
    sweep = {}
    for n in sorted({min(16, threads), min(64, threads), min(threads, 256)}):
        t0 = time.perf_counter()
        ob.pass_threaded(timed_passes, nthreads=n)
        sweep[n] = timed_passes * E / (time.perf_counter() - t0)
    best = max(sweep, key=sweep.get)
    hc = host_cpus()
    # cores: the CPU time the run could get -- the cgroup quota when one caps
    # the affinity set (16 of 256 on the GPU box), else the affinity set;
    # threads: the pool that ran the best pass (more threads than the quota
    # still overlap memory stalls); the machine's count beside them
    quota = hc["cgroup_quota_cpus"]
    eff = min(hc["available"], int(-(-quota // 1))) if quota else hc["available"]
    return {"value": sweep[best], "unit": "events/s", "cores": eff, "cores_source":
            "cgroup CPU quota" if quota and eff < hc["available"] else "affinity set",
            "cores_visible": hc["available"], "threads": best,
            "thread_sweep": {str(k): round(v) for k, v in sweep.items()},
            "host_cpus": hc["machine"], "cgroup_quota_cpus": hc["cgroup_quota_cpus"], "kind": "port",
            "n_syn": n_syn, "graph": ("reduced: %d of %d synapses, picks hit a smaller working set than "
                                      "the GPU's (likely overstates the CPU rate)" % (n_syn, wl.n_syn))
            if reduced else "same records as the GPU run",
            "sample": f"{what}, {wl.n_neuron:,} neurons, {settle} untimed + {timed_passes} timed passes, "
                      f"oracle_pass_threaded, best of {sorted(sweep)} threads on {hc['available']} CPUs "
                      f"(cgroup quota {hc['cgroup_quota_cpus']} CPUs)"}


def raw_run(config: str, events_arg: int, settle: int, warmup: int, steps: int, clock_passes: int = 0) -> dict:
    """One step = one pass of abnn_launch_traversal over caller-owned
    buffers in the reference's layouts (brain.cpp:52-69): the host's two
    writes of encode_traversal / inject_inputs (lastF[inputs] = clock,
    budget = kMaxSpikes; brain.cpp:82,90) as two tiny torch kernels, then
    the launcher's kernels.  The record buffer holds all N_SYN records (16 GB
    at config 3); its first E (the only ones a sweep reads) are the
    build_random_graph recipe generated on the GPU by the handle API."""
    import ctypes as C

    import torch

    from abnn_amd import CONFIGS, Brain, _lib

    wl = CONFIGS[config]
    events = events_arg or wl.events
    E = min((events + 255) // 256 * 256, wl.n_syn)
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    gen = Brain(wl.n_input, wl.n_output, wl.n_hidden, E, events, device=0)
    gen.build_random_graph(1)
    head = gen.download_synapses(0, E)
    del gen
    recs = torch.zeros((wl.n_syn, 4), dtype=torch.int32, device=dev)
    recs[:E].copy_(torch.from_numpy(head.view(np.int32).reshape(-1, 4)))
    del head
    n_nrn = wl.n_neuron
    lastF = torch.zeros(n_nrn, dtype=torch.int32, device=dev)
    lastV = torch.zeros(n_nrn, dtype=torch.int32, device=dev)
    scal = torch.zeros(4, dtype=torch.int32, device=dev)  # clock, budget, reward, rBar
    nb = int(lib.abnn_traversal_workspace_bytes(wl.n_syn, events))
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    kp = _lib.default_params()
    a = _lib.TraversalArgs()
    p = scal.data_ptr()
    a.syn, a.last_fired, a.last_visited, a.clock = recs.data_ptr(), lastF.data_ptr(), lastV.data_ptr(), p
    a.n_syn, a.tau_vis, a.tau_pre = wl.n_syn, 50_000, 50_000
    a.a_ltp, a.a_ltd, a.w_min, a.w_max = kp.a_ltp, kp.a_ltd, kp.w_min, kp.w_max
    a.budget, a.reward, a.rbar = p + 4, p + 8, p + 12
    a.n_nrn, a.events, a.knobs = n_nrn, events, None
    a.workspace, a.workspace_bytes = ws.data_ptr(), nb

    def step(n: int) -> None:
        for _ in range(n):
            lastF[:wl.n_input] = scal[0]             # inject_inputs, every input firing (brain.cpp:82)
            scal[1:2].fill_(int(kp.max_spikes))      # encode_traversal resets the budget (brain.cpp:90);
                                                     # a device fill, not a 4-B host copy per pass
            if lib.abnn_launch_traversal(C.byref(a), None) != 0:
                raise RuntimeError("abnn_launch_traversal failed")

    ts = time.perf_counter()
    step(settle)
    torch.cuda.synchronize()
    settle_s = time.perf_counter() - ts
    step(warmup)
    torch.cuda.synchronize()
    g = (C.c_uint64 * 2)()
    lib.abnn_debug_raw_gate_timing(1)
    ev_a, ev_b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g1 = g2 = 0
    t0 = time.perf_counter()
    ev_a.record()
    step(steps)
    ev_b.record()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    lib.abnn_debug_raw_stats(ws.data_ptr(), g, None)  # the last pass's
    g1, g2 = int(g[0]), int(g[1])
    clk = []
    for _ in range(clock_passes):  # untimed passes, each one's per-wave timeline (tools/raw_clock.py)
        step(1)
        c = np.zeros(8 * 4096, dtype=np.uint64)
        lib.abnn_debug_raw_wave_clock(ws.data_ptr(), nb, wl.n_syn, events,
                                      c.ctypes.data_as(C.POINTER(C.c_uint64)), c.size, None)
        clk.append(c.reshape(4096, 8))
    gate_ms, n_gate = C.c_double(), C.c_uint32()
    lib.abnn_debug_raw_gate_time(C.byref(gate_ms), C.byref(n_gate))
    lib.abnn_debug_raw_gate_timing(0)
    region_ms = float(ev_a.elapsed_time(ev_b))
    avg_gate_ms = gate_ms.value / max(1, n_gate.value)
    stream_bytes = 16 * E
    achieved = stream_bytes / (avg_gate_ms * 1e-3) / 1e9
    # SURVEY §8(d) for the reference's own accesses, u32 timestamps (VERDICT r3
    # item 3): 16 B record + 4 B lastF[src] per event, 4 B lastF[dst] per
    # pre-gated event (+ 16 B per update and 4 B per spike, not counted: the
    # update/stamp kernels, < 0.1 % of the bytes at config 3)
    survey = 20 * E + 4 * g1
    # the fused pass (k_raw_pass: the gate, the budget, the walk and the
    # stamps in one launch after k_raw_filter) or round 4's five launches
    kname = "k_raw_pass" if lib.abnn_debug_raw_fused_active() else "k_raw_gate"
    traffic, traffic_note = load_traffic("raw_" + wl.name)
    if traffic and traffic.get("kernel") != kname:
        traffic, traffic_note = None, "profiles/traffic_raw_%s.json is of %s, this run's kernel is %s" % (
            wl.name, traffic.get("kernel"), kname)
    out = {
        "metric": "traversal events/sec at 1B synapses, 5M neurons; achieved HBM GB/s",
        "value": E * steps / dt, "unit": "events/s", "n_gpus": 1, "steps": steps,
        "warmup": warmup, "ms_per_step": dt / steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (build_random_graph recipe, portable RNG, generated on GPU)",
        "config": {"workload": f"{wl.name} reference layout: abnn_launch_traversal over caller-owned "
                               f"16-B records ({wl.n_syn:,} x 16 B) and u32 lastF",
                   "n_neuron": n_nrn, "n_syn": wl.n_syn, "visited_events_per_pass": E,
                   "workspace_bytes": nb, "settle_passes": settle, "settle_s": round(settle_s, 3),
                   "last_pass_pre_gated": g1, "last_pass_survivors": g2,
                   "host_writes_per_pass": "lastF[inputs] = clock, budget = kMaxSpikes (2 torch kernels)"},
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic.get("bytes_per_launch") if traffic else None,
            "traffic_stream_bytes": traffic.get("stream_bytes") if traffic else None,
            "traffic_other_fetch_bytes": traffic.get("other_fetch_bytes") if traffic else None,
            "traffic_source": ("profiles/traffic_raw_%s.json (rocprofv3 PMC of %s: the record stream from "
                               "FETCH_SIZE x2, the rest of FETCH_SIZE x1, + WRITE_SIZE, calibrated by "
                               "profiles/r05_fetch_calibration.txt; tag %s, kernel sources %s)"
                               % (wl.name, kname, traffic.get("tag"), traffic.get("source_sha"))
                               if traffic else traffic_note),
            "kernel": kname, "avg_launch_ms": round(avg_gate_ms, 4), "timed_launches": n_gate.value,
            "launch_ms_source": "HIP event pair around every %s launch (abnn_debug_raw_gate_timing)" % kname,
            "algorithmic_bytes_per_launch": stream_bytes,
            "bytes_formula": "16*E (the caller's 16-B SynapsePacked record per visited event; DESIGN.md §5)",
            "survey_formula_bytes_per_launch": survey,
            "survey_formula_achieved": round(survey / (avg_gate_ms * 1e-3) / 1e9, 1),
            "survey_formula": "20*E + 4*G1 (SURVEY §8d with u32 lastF: record + lastF[src] per event, "
                              "lastF[dst] per pre-gated; G1 of the last pass)",
            "pass_ms_events": round(region_ms / steps, 4),
        },
        "cpu_baseline": None,
    }
    if clk:
        out["_wave_clocks"] = np.stack(clk)
    del recs, ws, lastF, lastV
    torch.cuda.empty_cache()
    return out


def raw_main(args) -> None:
    """--raw: the reference-layout path (raw_run) as the bench line itself."""
    out = raw_run(args.config, args.events, args.settle, args.warmup, args.steps)
    print(json.dumps(out), file=_JSON_OUT, flush=True)


def reference_layout_summary(config: str, settle: int) -> dict:
    """The drop-in path over the reference's own buffers (abnn_launch_traversal,
    16-B records), timed in the same run as the headline line: its pass and
    gate times and its roofline on 16 B per visited event."""
    r = raw_run(config, 0, settle, 10, 50)
    rf = r["roofline"]
    return {"api": "abnn_launch_traversal (caller-owned 16-B SynapsePacked records, u32 lastF; brain.metal:42-58)",
            "events_per_s": r["value"], "pass_ms": round(r["ms_per_step"], 4), "steps": r["steps"],
            "gate_kernel": rf["kernel"], "gate_ms": rf["avg_launch_ms"], "gate_timed_launches": rf["timed_launches"],
            "bytes_per_pass": rf["algorithmic_bytes_per_launch"], "bytes_formula": rf["bytes_formula"],
            "achieved_gbs": rf["achieved"], "frac": rf["frac"], "traffic": rf["traffic"],
            "traffic_source": rf["traffic_source"], "pass_ms_events": rf["pass_ms_events"]}


_JSON_OUT = sys.stdout


def main():
    args = parse()
    # stdout carries the ONE JSON line: anything else the process prints on
    # file descriptor 1 (RCCL's init banner, runtime notices) goes to stderr
    sys.stdout.flush()
    global _JSON_OUT
    _JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    if args.raw:
        if int(os.environ.get("WORLD_SIZE", "1")) != 1:
            raise SystemExit("--raw runs on one GPU")
        raw_main(args)
        return
    import torch

    from abnn_amd import CONFIGS, Brain
    from abnn_amd.shard import ShardedBrain, TorchComm

    wl = CONFIGS[args.config]
    mode = 1 if args.mode == "random" else 0
    events = args.events or wl.events
    extra = dict(PLASTICITY) if args.plasticity else {}
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dist = None
    # one GPU per rank; ABNN_DIST_BACKEND=gloo rehearses the multi-rank path with
    # ranks sharing the visible GPUs (exchange tensors staged through the host)
    backend = os.environ.get("ABNN_DIST_BACKEND", "nccl")
    device = local_rank if backend == "nccl" else local_rank % max(1, torch.cuda.device_count())
    if world == 1 and args.shard_path:  # a one-rank process group for the sharded path
        import socket

        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            with socket.socket() as so:
                so.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(so.getsockname()[1])
        dist.init_process_group("gloo", rank=0, world_size=1)
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(device)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)

    if world > 1 or args.shard_path:
        # one GPU per rank (RCCL): the passes are driven by the C-ABI over the
        # library's RCCL communicator (abnn_shard_traverse); the gloo
        # rehearsal (ranks sharing a GPU) drives them phase by phase from Python
        sb = ShardedBrain(TorchComm(), wl.n_input, wl.n_output, wl.n_hidden, wl.n_syn, events,
                          device=device, mode=mode, capacity_factor=1.01 if args.plasticity else 1.0,
                          native=backend == "nccl" or world == 1, **extra)
        brain = sb.brain
        step = sb.step
    else:
        cap = int(wl.n_syn * 1.01) if args.plasticity else 0
        brain = Brain(wl.n_input, wl.n_output, wl.n_hidden, wl.n_syn, events, device=device, mode=mode,
                      syn_capacity=cap, **extra)
        step = brain.encode_traversal
    brain.build_random_graph(1)
    brain.set_auto_stimulus(0, wl.n_input)
    if args.plasticity:
        brain.set_reward(0.25)  # reward-modulated STDP active (MSL:105-107)
    local_events = brain.visited_events()

    def sync():
        brain.synchronize()
        torch.cuda.synchronize(device)
        if dist is not None:
            dist.barrier()

    # start-up transient (untimed): the freshly built graph to its steady state
    ts = time.perf_counter()
    step(args.settle)
    sync()
    settle_s = time.perf_counter() - ts
    step(args.warmup)
    sync()
    brain.reset_stats()
    sync()
    # one HIP event pair around the K timed passes, on the stream they are
    # enqueued on (the device's null stream = torch's default stream): the
    # average launch duration is its span / K (one k_gate launch per pass in
    # steady state; the ~1 us dispatch gap between launches included)
    ev_a, ev_b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev_a.record()
    step(args.steps)
    ev_b.record()
    # the contract's closing bracket: a device-wide synchronize (it covers the
    # brain's stream, torch's default one) and, across ranks, the barrier.
    # brain.synchronize() -- the same wait once more, plus its error check --
    # runs after the clock stops: a second host wake-up was ~1 us per pass of
    # a 20-pass driver run
    torch.cuda.synchronize(device)
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    brain.synchronize()
    region_ms = float(ev_a.elapsed_time(ev_b))
    stats = brain.stats()
    # then, untimed: an event pair around a sample of single launches (every
    # TIMING_EVERY-th; a pair adds a few us to the launch it brackets) for
    # the min / median and the steady-state check
    every = timing_every(args.steps)
    brain.enable_timing(every)
    step(args.steps)
    sync()
    launch_ms = brain.kernel_times()
    launches = int(launch_ms.size)
    brain.enable_timing(0)
    if dist is not None:
        tdev = f"cuda:{device}" if backend == "nccl" else "cpu"
        t = torch.tensor([dt], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        ev = torch.tensor([stats["events"]], dtype=torch.float64, device=tdev)
        dist.all_reduce(ev, op=dist.ReduceOp.SUM)
        total_events = float(ev.item())
    else:
        total_events = float(stats["events"])

    if rank == 0:
        value = total_events / dt
        avg_gate_ms = region_ms / args.steps
        track = bool(brain.params.track_visits)
        # one gate launch per pass; HIP events time a sample of them (every
        # TIMING_EVERY-th), so bytes per launch come from the pass count
        passes = max(1, stats["passes"])
        bytes_per_launch = algorithmic_bytes(stats, track, mode == 1) / passes
        achieved = bytes_per_launch / (avg_gate_ms * 1e-3) / 1e9
        survey_per_launch = survey_bytes(stats, track) / passes
        default_run = mode == 0 and events == wl.events and not args.shard_path
        traffic, traffic_note = load_traffic(args.config) if world == 1 and default_run else (None, "not the default run")
        roofline = {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic.get("bytes_per_launch") if traffic else None,
            "traffic_stream_bytes": traffic.get("stream_bytes") if traffic else None,
            "traffic_other_fetch_bytes": traffic.get("other_fetch_bytes") if traffic else None,
            "kernel": "k_gate", "avg_launch_ms": round(avg_gate_ms, 4), "timed_launches": args.steps,
            "launch_ms_source": "HIP event pair around the timed passes / steps (launch + dispatch gap)",
            "sampled_launches": launches,
            "sampled_min_launch_ms": round(float(launch_ms.min()), 4) if launches else None,
            "sampled_median_launch_ms": round(float(np.median(launch_ms)), 4) if launches else None,
            "timing_every": every,
            # a launch cannot take longer than the pass it is part of: if the
            # sample's median says so (beyond the few us an event pair adds to
            # the launch it brackets), the timed window still held the transient
            "steady": bool(launches and float(np.median(launch_ms)) <= 1.08 * dt / args.steps * 1e3),
            "algorithmic_bytes_per_launch": int(bytes_per_launch),
            "bytes_formula": ("3*E (24-bit src stream: 2-B lo + 1-B hi per event; E visited events) -- "
                              "DESIGN.md §5" if mode == 0 else
                              "64*E (one random 64-B HBM line per pick of the src32 mirror; 4 B of it "
                              "used) -- DESIGN.md §5"),
            "random_picks_per_s": (round(stats["events"] / passes / (avg_gate_ms * 1e-3), 1) if mode == 1 else None),
            "survey_formula_bytes_per_launch": int(survey_per_launch),
            "survey_formula_achieved": round(survey_per_launch / (avg_gate_ms * 1e-3) / 1e9, 1),
            "survey_formula": "24*E + 8*G1 (SURVEY §8d; G1 pre-gated) -- counts an 8-B lastFired[src] "
                              "gather per event that this design answers from LDS/L2",
            "traffic_source": ("profiles/traffic_%s.json (rocprofv3 PMC of k_gate: the 3-B/event stream from "
                               "FETCH_SIZE x2, the rest of FETCH_SIZE x1, + WRITE_SIZE, calibrated by "
                               "profiles/r05_fetch_calibration.txt; tag %s, kernel sources %s)"
                               % (args.config, traffic.get("tag"), traffic.get("source_sha"))
                               if traffic else traffic_note),
            "pass_ms": round(dt / args.steps * 1e3, 4),
        }
        ref_layout = None
        if world == 1 and default_run and not args.plasticity and not args.no_reference_layout:
            brain.close()  # its device memory before the reference-layout buffers (16 GB of records)
            del step, brain
            torch.cuda.empty_cache()
            ref_layout = reference_layout_summary(args.config, args.settle)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            avail = host_cpus()["available"]
            threads = avail if args.cpu_threads <= 0 else max(1, min(args.cpu_threads, avail))
            # random mode on the CPU is ~100x slower per pass: 6 settle passes
            cpu = cpu_baseline(wl, events, mode, threads, args.cpu_passes, extra,
                               args.settle if mode == 0 else min(args.settle, 6))
        out = {
            "metric": "traversal events/sec at 1B synapses, 5M neurons; achieved HBM GB/s",
            "value": value, "unit": "events/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (build_random_graph recipe, portable RNG, generated on GPU)",
            "config": {
                "workload": f"{wl.name}: {wl.note}; " + (f"sharded {world} ways, one GPU per shard" if world > 1
                                                         else "one GPU holds the whole graph"), "n_neuron": wl.n_neuron, "n_syn": wl.n_syn,
                "events_per_pass_per_gpu": events, "visited_events_per_pass_per_gpu": local_events,
                "mode": args.mode,
                "plasticity": (dict(PLASTICITY, syn_capacity_factor=1.01, reward=0.25,
                                    n_syn_after=brain.n_syn(), pruned=stats.get("pruned", 0),
                                    grown=stats.get("grown", 0)) if args.plasticity else None),
                "parallelism": (f"synapse-shard dp{world}" + ("" if backend == "nccl" else f" ({backend} rehearsal)"))
                               if world > 1 else ("synapse-shard dp1 (the sharded pass at one GPU)" if args.shard_path
                                                  else "single GPU"),
                "settle_passes": args.settle, "settle_s": round(settle_s, 4),
                "pre_gated_frac": stats["pre_gated"] / max(1, stats["events"]),
                "spikes_per_pass": stats["fired"] / max(1, stats["passes"]),
            },
            "roofline": roofline, "cpu_baseline": cpu, "reference_layout": ref_layout,
        }
        print(json.dumps(out), file=_JSON_OUT, flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
