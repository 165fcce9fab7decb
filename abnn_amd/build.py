"""In-tree build of the HIP library (and, for the test harness, the oracle).

* ``build_hip()``    : hipcc --offload-arch=gfx950 -> abnn_amd/libabnn_hip.so
* ``build_oracle()`` : gcc -> oracle/liboracle.so (test infrastructure)
* ``build_cpp_example()`` : g++ -> tests/cpp/brain_cpp_test (C++ Brain API over the C-ABI)

All fp32 code is compiled with -ffp-contract=off so that the GPU and the CPU
oracle round every operation identically (bit-exact weights).
"""
from __future__ import annotations

import os
import shutil
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "abnn_amd")
CSRC = os.path.join(PKG, "csrc")
HIP_SOURCES = [os.path.join(CSRC, "kernels.hip"), os.path.join(CSRC, "capi.hip"), os.path.join(CSRC, "raw.hip")]
HIP_DEPS = HIP_SOURCES + [os.path.join(CSRC, "engine.h"), os.path.join(CSRC, "device.h"),
                          os.path.join(ROOT, "include", "abnn", "abnn.h")]
LIB = os.path.join(PKG, "libabnn_hip.so")
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "liboracle.so")
CPP_TEST_SRC = os.path.join(ROOT, "tests", "cpp", "brain_cpp_test.cpp")
CPP_TEST_BIN = os.path.join(ROOT, "tests", "cpp", "brain_cpp_test")
ENGINE_TEST_SRC = os.path.join(ROOT, "tests", "cpp", "engine_test.cpp")
ENGINE_TEST_BIN = os.path.join(ROOT, "tests", "cpp", "engine_test")
ENGINE_HOST_SRC = os.path.join(ROOT, "tests", "cpp", "engine_host_test.cpp")
ENGINE_HOST_BIN = os.path.join(ROOT, "tests", "cpp", "engine_host_test")

HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")
HIP_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
             "-ffp-contract=off", "-Wall", "-Werror=return-type", "-ldl"]


def kernel_source_sha() -> str:
    """sha256 (16 hex) of the HIP library's sources: ties a committed
    measurement (profiles/traffic_*.json) to the kernels it was taken on."""
    import hashlib

    h = hashlib.sha256()
    for p in sorted(HIP_DEPS):
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build_hip(force: bool = False, out: str | None = None, defines: list[str] | None = None) -> str:
    """The three translation units compiled in parallel (each ~20-60 s), then
    linked.  out / defines: an experiment build (tools/build_variant.sh)."""
    target = out or LIB
    if force or out or _stale(target, HIP_DEPS):
        comp = [f for f in HIP_FLAGS if f not in ("-shared", "-ldl")]
        objs, procs = [], []
        for src in HIP_SOURCES:
            obj = f"{target}.{os.path.basename(src)}.o"
            objs.append(obj)
            cmd = [HIPCC, *comp, *(defines or []), "-c", "-o", obj, src]
            procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)))
        errs = []
        for cmd, p in procs:
            o, e = p.communicate()
            if p.returncode != 0:
                errs.append(f"build failed ({p.returncode}): {' '.join(cmd)}\n{o}\n{e}")
        if errs:
            for obj in objs:
                if os.path.exists(obj):
                    os.remove(obj)
            raise RuntimeError("\n".join(errs))
        tmp = target + ".tmp"
        _run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp, *objs, "-ldl"])
        for obj in objs:
            os.remove(obj)
        os.replace(tmp, target)
    return target


def build_oracle(force: bool = False) -> str:
    src = os.path.join(ORACLE_DIR, "c1_oracle.c")
    deps = [src, os.path.join(ORACLE_DIR, "c1_oracle.h"), os.path.join(ROOT, "include", "abnn", "abnn.h")]
    if force or _stale(ORACLE_LIB, deps):
        tmp = ORACLE_LIB + ".tmp"
        _run(["gcc", "-O2", "-std=c11", "-Wall", "-ffp-contract=off", "-fPIC", "-shared",
              "-pthread", "-o", tmp, src])
        os.replace(tmp, ORACLE_LIB)
    return ORACLE_LIB


def build_cpp_example(force: bool = False) -> str | None:
    if not os.path.exists(CPP_TEST_SRC):
        return None
    deps = [CPP_TEST_SRC, LIB, os.path.join(ROOT, "include", "abnn", "brain.hpp")]
    if force or _stale(CPP_TEST_BIN, deps):
        _run(["g++", "-O2", "-std=c++17", "-Wall", "-I", os.path.join(ROOT, "include"),
              "-o", CPP_TEST_BIN, CPP_TEST_SRC, "-L", PKG, "-labnn_hip",
              f"-Wl,-rpath,{PKG}", "-Wl,-rpath,$ORIGIN/../../abnn_amd"])
    return CPP_TEST_BIN


def build_engine_tests(force: bool = False) -> tuple[str | None, str | None]:
    """Test programs of the learning driver (include/abnn/engine.hpp): the
    CPU-only known-answer program, and the GPU-vs-oracle driver run (links the
    oracle's C restatement -- test infrastructure, like the program itself)."""
    inc = os.path.join(ROOT, "include")
    hdrs = [os.path.join(inc, "abnn", "engine.hpp"), os.path.join(inc, "abnn", "brain.hpp")]
    host = None
    if os.path.exists(ENGINE_HOST_SRC):
        if force or _stale(ENGINE_HOST_BIN, [ENGINE_HOST_SRC, *hdrs]):
            _run(["g++", "-O2", "-std=c++17", "-Wall", "-ffp-contract=off", "-I", inc,
                  "-o", ENGINE_HOST_BIN, ENGINE_HOST_SRC])
        host = ENGINE_HOST_BIN
    gpu = None
    if os.path.exists(ENGINE_TEST_SRC):
        osrc = os.path.join(ORACLE_DIR, "c1_oracle.c")
        deps = [ENGINE_TEST_SRC, os.path.join(ROOT, "tests", "cpp", "oracle_brain.hpp"), osrc, LIB, *hdrs]
        if force or _stale(ENGINE_TEST_BIN, deps):
            obj = ENGINE_TEST_BIN + ".oracle.o"
            _run(["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-pthread", "-c", "-o", obj, osrc])
            _run(["g++", "-O2", "-std=c++17", "-Wall", "-ffp-contract=off", "-pthread", "-I", inc,
                  "-o", ENGINE_TEST_BIN, ENGINE_TEST_SRC, obj, "-L", PKG, "-labnn_hip",
                  f"-Wl,-rpath,{PKG}", "-Wl,-rpath,$ORIGIN/../../abnn_amd"])
            os.remove(obj)
        gpu = ENGINE_TEST_BIN
    return host, gpu


def build_all(force: bool = False) -> None:
    build_hip(force)
    build_oracle(force)
    build_cpp_example(force)
    build_engine_tests(force)


if __name__ == "__main__":
    build_all(force=True)
    print("built", LIB, ORACLE_LIB)
