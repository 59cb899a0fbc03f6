"""Build the native libraries in-tree.

* ``lib/libdml_hip.so`` — every HIP kernel (``csrc/kernels/*.hip``), compiled for
  gfx950 only (CDNA4 / MI355X).  hipcc cross-compiles without a GPU.
* ``lib/libdml_cpu.so`` — the C++ runtime (``csrc/runtime/*.cpp``): CPU tree builder,
  scheduler core, binning; g++ with OpenMP and ``-ffp-contract=off`` so split scores
  match the GPU builder bit-for-bit.

Usage: ``python -m cs230_distributed_machine_learning_amd.build [--force]``.
"""
from __future__ import annotations

import argparse
import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "lib")
HIP_LIB = os.path.join(LIB, "libdml_hip.so")
CPU_LIB = os.path.join(LIB, "libdml_cpu.so")
ARCH = os.environ.get("DML_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc"), shutil.which("hipcc") or ""):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the HIP kernels)")


def _stale(target: str, sources: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd: list[str]) -> None:
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        sys.stderr.write(res.stdout + res.stderr)
        raise RuntimeError(f"build failed: {' '.join(cmd)}")


def build_hip(force: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    deps = srcs + glob.glob(os.path.join(CSRC, "kernels", "*.h"))
    os.makedirs(LIB, exist_ok=True)
    if force or _stale(HIP_LIB, deps):
        tmp = HIP_LIB + ".tmp"
        _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
              "-Wno-unused-result", "-I", os.path.join(CSRC, "kernels"), *srcs, "-o", tmp])
        os.replace(tmp, HIP_LIB)
    return HIP_LIB


def build_cpu(force: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    deps = srcs + glob.glob(os.path.join(CSRC, "runtime", "*.h")) + glob.glob(os.path.join(CSRC, "kernels", "*.h"))
    os.makedirs(LIB, exist_ok=True)
    if force or _stale(CPU_LIB, deps):
        cxx = os.environ.get("CXX", shutil.which("g++") or "c++")
        tmp = CPU_LIB + ".tmp"
        _run([cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-fopenmp", "-ffp-contract=off",
              "-I", os.path.join(CSRC, "kernels"), *srcs, "-o", tmp])
        os.replace(tmp, CPU_LIB)
    return CPU_LIB


def build_all(force: bool = False) -> tuple[str, str]:
    return build_cpu(force), build_hip(force)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--cpu-only", action="store_true")
    args = ap.parse_args()
    print(build_cpu(args.force))
    if not args.cpu_only:
        print(build_hip(args.force))
