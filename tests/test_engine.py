"""The per-pass learning driver (include/abnn/engine.hpp ~ BrainEngine,
abnn/src/core/brain-engine.cpp:108-190).

CPU: the rate filter (rate-filter.h:22-59) and the sinusoid dataset
(functional-dataset.cpp:24-52) against an independent numpy restatement that
keeps the reference's float/double types (libm's cosf/sinf via ctypes, so the
transcendental values are the same library's).
GPU: the driver over the GPU brain vs the same driver over the CPU oracle --
outputs and normalised rates every pass, loss/reward every window, final
weights, lastFired, clock and rBar, bit for bit.  The reference seeds its
teacher RNG from random_device, so parity with the reference's own runs is
unpinned; this pins the GPU path against the oracle under the same seed."""
import ctypes
import ctypes.util
import json
import math
import subprocess

import numpy as np
import pytest

from abnn_amd.build import build_engine_tests

_libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
for _f in ("cosf", "sinf"):
    getattr(_libm, _f).restype = ctypes.c_float
    getattr(_libm, _f).argtypes = [ctypes.c_float]
F32 = np.float32


def _cos2(x):
    c = F32(_libm.cosf(F32(x)))
    return F32(c * c)


def _half_sine(x):
    return F32(F32(0.5) * F32(_libm.sinf(F32(x))) + F32(0.5))


def _frames(n=8, frames=12, dt=0.0009, hz=0.5):
    phase = t = 0.0
    two_pi = 2.0 * 3.14159265358979323846
    for _ in range(frames):
        phase += hz * dt
        if phase > 1.0:
            phase -= 1.0
        t += dt
        xin = [_cos2(np.float32(two_pi * (i / n + phase))) for i in range(n)]
        xex = [_half_sine(np.float32(two_pi * (i / n + phase))) for i in range(n)]
        yield np.array(xin, F32), np.array(xex, F32), t


class _Filter:
    def __init__(self, tau, fir, size=20):
        self.tau, self.fir, self.size = tau, fir, size
        self.state, self.hist = None, []

    def process(self, raw, dt):
        if self.state is None:
            self.state = raw.copy()
        a = dt / (self.tau + dt)
        self.state = (self.state + (a * (raw - self.state).astype(np.float64)).astype(F32)).astype(F32)
        if not self.fir:
            return self.state.copy()
        self.hist.append(self.state.copy())
        if len(self.hist) > self.size:
            self.hist.pop(0)
        acc = np.zeros_like(raw)
        for f in self.hist:
            acc = (acc + f).astype(F32)
        return (acc * (F32(1) / F32(len(self.hist)))).astype(F32)


def test_rate_filter_and_dataset_known_answers():
    host, _ = build_engine_tests()
    out = json.loads(subprocess.run([host], capture_output=True, text=True, check=True).stdout)
    iir, fir = _Filter(0.02, False), _Filter(0.02, True, 5)
    t_end = 0.0
    for f, (xin, xex, t) in enumerate(_frames()):
        raw = np.array([((f * 7 + i * 3) % 5) * 0.25 for i in range(8)], F32)
        got = out["frames"][f]
        assert np.array_equal(np.array(got["in"], F32), xin), f
        assert np.array_equal(np.array(got["ex"], F32), xex), f
        assert np.array_equal(np.array(got["iir"], F32), iir.process(raw, 0.0009)), f
        assert np.array_equal(np.array(got["fir"], F32), fir.process(raw, 0.0009)), f
        t_end = t
    assert math.isclose(out["time"], t_end, rel_tol=0, abs_tol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("passes,win", [(300, 50), (2100, 1000)])
def test_driver_gpu_matches_oracle(gpu, passes, win):
    _, prog = build_engine_tests()
    r = subprocess.run([prog, str(passes), str(win)], capture_output=True, text=True, timeout=600)
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0 and res["ok"], (res, r.stderr[-2000:])
    assert res["windows"] == passes // win
    assert res["spikes"] > 0
