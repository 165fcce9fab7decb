"""Independent pure-Python restatement of brain.metal for SMALL cases.

Test infrastructure: written as an emulator of the Metal kernel's threads
(abnn/src/core/kernels/brain.metal:41-130) rather than as the C1 loop of the C
oracle, so the two restatements can check each other.  Metal relaxed atomics
are modelled as "cells": every load of lastF / clock / rBar returns the value
at kernel start (schedule C1), stores land in a pending set applied when the
kernel ends; the budget cell is sequentially consistent in tid order.  fp32
arithmetic uses numpy.float32 scalars so every operation rounds to fp32 on its
own (the C oracle and the HIP kernels are built with -ffp-contract=off).
"""
from __future__ import annotations

import numpy as np

F = np.float32
U32 = 0xFFFFFFFF
U64 = 0xFFFFFFFFFFFFFFFF


def rand01(s: int) -> np.float32:
    s &= U32
    s ^= (s << 13) & U32
    s ^= s >> 17
    s ^= (s << 5) & U32
    return F(s & 0xFFFFFF) * F(1.0 / 16777216.0)


def metal_clamp(x, lo, hi):
    return min(max(x, lo), hi)


class Cell:
    """A device atomic with deferred visibility (C1)."""

    def __init__(self, v):
        self.v = v
        self.pending = None

    def load(self):
        return self.v

    def store(self, v):
        self.pending = v

    def commit(self):
        if self.pending is not None:
            self.v, self.pending = self.pending, None


M32 = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    """Philox4x32-10 (Salmon et al., SC'11), written independently of the C oracle."""
    x0, x1, x2, x3 = ctr
    k0, k1 = key
    for _ in range(10):
        p0, p1 = 0xD2511F53 * x0, 0xCD9E8D57 * x2
        x0, x1, x2, x3 = ((p1 >> 32) ^ x1 ^ k0) & M32, p1 & M32, ((p0 >> 32) ^ x3 ^ k1) & M32, p0 & M32
        k0, k1 = (k0 + 0x9E3779B9) & M32, (k1 + 0xBB67AE85) & M32
    return x0, x1, x2, x3


def pick(seed, stream, pass_index, t, n_syn):
    """Random-mode record of event t (include/abnn/abnn.h)."""
    k = seed ^ stream
    o = philox4x32_10((t & M32, t >> 32, pass_index & M32, pass_index >> 32), (k & M32, k >> 32))
    return (((o[1] << 32) | o[0]) * n_syn) >> 64


U64M = (1 << 64) - 1
GENESIS_KEY = 0xA24BAED4963EE407
TOMB = 0xFFFFFFFF


def splitmix64_at(seed, k):
    z = (seed + ((k + 1) * 0x9E3779B97F4A7C15)) & U64M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & U64M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & U64M
    return z ^ (z >> 31)


class MetalEmu:
    """State of one Brain: synapse list, lastFired cells, scalars."""

    def __init__(self, syn_src, syn_dst, syn_w, n_nrn, events, params):
        self.src = [int(x) for x in syn_src]
        self.dst = [int(x) for x in syn_dst]
        self.w = [F(x) for x in syn_w]
        self.lastF = [0] * n_nrn
        self.lastV = [0] * n_nrn
        self.clock = 0
        self.reward = F(0.0)
        self.rbar = F(0.0)
        self.events = int(events)
        self.p = params
        self.stim = (0, 0)
        self.pass_index = 0
        self.n_in = 256
        self.capacity = len(self.src)
        self.grown = {}  # slot -> (src, dst, w) grown since the last structural update
        self.pruned = 0
        self.n_grown = 0

    def kernel(self):
        """One dispatch of monte_carlo_traversal over roundup(EVENTS,256) threads
        (sweep), or EVENTS threads each visiting a random record (random mode:
        every thread reads the pass-start record; stores land in tid order)."""
        p = self.p
        n_syn = len(self.src)
        random = p.get("mode", 0) == 1
        grid = self.events if random else (self.events + 255) // 256 * 256
        w0 = list(self.w)
        rec = [pick(p["seed"], 0, self.pass_index, t, n_syn) for t in range(grid)] if random and n_syn else None
        lastF = [Cell(v) for v in self.lastF]
        clock = Cell(self.clock)
        rbar = Cell(self.rbar)
        budget = p["max_spikes"]   # host reset, brain.cpp:90 (sequentially consistent)
        now_tg = clock.load()      # every TG caches the same pass-start value under C1
        ticked = False
        stores = []
        visit_dst = ([self.dst[rec[t] if random else t] for t in range(grid if random else min(grid, n_syn))]
                     if p.get("track_visits") else None)
        for tid in range(grid):
            if not random and tid >= n_syn:
                break                               # brain.metal:61
            if random and n_syn == 0:
                break
            e = rec[tid] if random else tid
            now = now_tg
            if self.src[e] == TOMB:
                ticked |= tid == 0
                continue                            # removed synapse (README §5)
            lp = lastF[self.src[e]].load()
            if (now - lp) & U32 > p["window_pre"]:   # uint arithmetic, MSL:74
                ticked |= tid == 0
                continue
            ld = lastF[self.dst[e]].load()
            if (now - ld) & U32 <= p["refractory"]:  # MSL:80
                ticked |= tid == 0
                continue
            if budget == 0:
                ticked |= tid == 0
                continue
            w = w0[e]
            prob = metal_clamp(F(w * w) * F(p["base_scale"]), F(0.0), F(1.0))
            fired = prob > rand01((tid & U32) ^ (now & U32))
            slot = None
            if fired:
                old = budget
                budget -= 1
                if old == 0:
                    fired = False
                else:
                    slot = p["max_spikes"] - old    # budget position of this spike
            dW = F(F(p["a_ltp"]) * F(F(1.0) - w)) if fired else F(F(-p["a_ltd"]) * w)
            R = self.reward
            rb = rbar.load()
            dW = F(dW + F(F(F(p["eta_reward"]) * F(R - rb)) * F(1.0 if fired else 0.0)))
            if tid == 0:
                rbar.store(F(rb + F(F(p["alpha_rbar"]) * F(R - rb))))
            isi = F((now - ld) & U32)                # float(uint), MSL:116
            est = F(F(1e6) / isi) if isi > F(0.0) else F(0.0)
            dW = F(dW + F(F(F(p["eta_home"]) * F(F(p["target_rate_hz"]) - est)) * w))
            nw = metal_clamp(F(w + dW), F(p["w_min"]), F(p["w_max"]))
            stores.append((e, nw))                  # applied after the sweep, last writer wins
            if fired:
                lastF[self.dst[e]].store(now)
                if p.get("p_new", 0) > 0 and p.get("compact_every", 0) > 0:
                    x = splitmix64_at(p["seed"] ^ GENESIS_KEY, ((self.pass_index << 32) | slot) & U64M)
                    if F(F(x >> 40) * F(1.0 / 16777216.0)) < F(p["p_new"]):
                        span = len(self.lastF) - self.n_in
                        dst2 = self.n_in + (((x & U32) * span) >> 32)
                        self.grown[(self.pass_index % p["compact_every"]) * p["max_spikes"] + slot] = (
                            self.src[e], dst2, F(p["w_init"]))
            ticked |= tid == 0
        last = {}
        for e, nw in stores:
            last[e] = nw
        for e, nw in last.items():
            self.w[e] = nw
            if p.get("w_prune", 0) > 0 and nw < F(p["w_prune"]):
                self.src[e] = self.dst[e] = TOMB
                self.pruned += 1
        for c in lastF:
            c.commit()
        rbar.commit()
        self.lastF = [c.v for c in lastF]
        self.rbar = rbar.v
        if ticked:
            self.clock = (now_tg + p["clock_inc"]) & U64
        if p.get("track_visits"):
            for tid in range(grid if random else min(grid, n_syn)):
                dv = visit_dst[tid]
                if dv != TOMB:
                    self.lastV[dv] = now_tg
        self.pass_index += 1
        ce = p.get("compact_every", 0)
        if ce and self.pass_index % ce == 0:          # structural update (abnn.h contract)
            # the array shrinks to m = n - D: the tombstones below m, in
            # order, take the live records of the tail [m, n), in order
            D = sum(1 for x in self.src if x == TOMB)
            if D:
                m = len(self.src) - D
                recs = list(zip(self.src, self.dst, self.w))
                fill = iter([r for r in recs[m:] if r[0] != TOMB])
                recs = [next(fill) if r[0] == TOMB else r for r in recs[:m]]
                self.src = [r[0] for r in recs]
                self.dst = [r[1] for r in recs]
                self.w = [r[2] for r in recs]
            for slot in sorted(self.grown):
                if len(self.src) < self.capacity:
                    s_, d_, w_ = self.grown[slot]
                    self.src.append(s_)
                    self.dst.append(d_)
                    self.w.append(w_)
                    self.n_grown += 1
            self.grown = {}

    def one_pass(self):
        """run_one_pass minus the host driver: stimulus, kernel, renorm (brain.cpp:87-141)."""
        first, count = self.stim
        for i in range(first, first + count):
            self.lastF[i] = self.clock
        renorm = (self.clock & U32) > self.p["renorm_thresh"]   # host read (u32) before the pass
        self.kernel()
        if renorm:                                      # brain.metal:135-145
            base = self.clock
            self.lastF = [(v - base) & U64 for v in self.lastF]
            self.clock = 0
