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


def _portable_flag(f: str) -> str:
    """A flag as it enters the content hash: paths relative to the package, a compiler by
    basename -- a tree moved to another path (the GPU box's scratch copy) hashes the same."""
    if os.path.isabs(f):
        return os.path.relpath(f, CSRC) if f.startswith(CSRC) else os.path.basename(f)
    return f


_VERSIONS: dict = {}


def _compiler_version(exe: str) -> str:
    if exe not in _VERSIONS:
        try:
            out = subprocess.run([exe, "--version"], capture_output=True, text=True, timeout=60).stdout
            _VERSIONS[exe] = out.splitlines()[0] if out else ""
        except Exception:
            _VERSIONS[exe] = ""
    return _VERSIONS[exe]


def _src_hash(sources: list[str], flags: list[str]) -> str:
    import hashlib

    h = hashlib.sha256(" ".join(_portable_flag(f) for f in flags).encode())
    for f in flags[:1]:   # the compiler (first flag for the C++ builds) by version, not by path
        if os.path.isabs(f) and os.path.exists(f):
            h.update(_compiler_version(f).encode())
    for s in sorted(sources, key=lambda p: os.path.relpath(p, CSRC)):
        with open(s, "rb") as f:
            h.update(os.path.relpath(s, CSRC).encode() + b"\0" + f.read())
    return h.hexdigest()


class _BuildLock:
    """An exclusive fcntl lock on ``lib/.build.lock``: ranks that start together (torchrun)
    check staleness, build and stamp one at a time -- the first builds, the rest find the
    stamp current and load the finished library."""

    def __enter__(self):
        import fcntl

        os.makedirs(LIB, exist_ok=True)
        self.f = open(os.path.join(LIB, ".build.lock"), "w")
        fcntl.flock(self.f, fcntl.LOCK_EX)
        return self

    def __exit__(self, *a):
        import fcntl

        fcntl.flock(self.f, fcntl.LOCK_UN)
        self.f.close()
        return False


def _tmp(out: str) -> str:
    return f"{out}.{os.getpid()}.tmp"


def _stale_by_hash(target: str, sources: list[str], flags: list[str]) -> bool:
    """Content-keyed staleness (a fresh checkout gives every file a new mtime, so an
    mtime test can pick a stale executable): the build stores the hash of its sources
    and flags next to the target."""
    stamp = target + ".srchash"
    if not os.path.exists(target) or not os.path.exists(stamp):
        return True
    with open(stamp) as f:
        return f.read().strip() != _src_hash(sources, flags)


def _stamp(target: str, sources: list[str], flags: list[str]) -> None:
    with open(target + ".srchash", "w") as f:
        f.write(_src_hash(sources, flags))


def _run(cmd: list[str]) -> None:
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        sys.stderr.write(res.stdout + res.stderr)
        raise RuntimeError(f"build failed: {' '.join(cmd)}")


def build_hip(force: bool = False, out: str = HIP_LIB, extra_flags: tuple = ()) -> str:
    """``out`` / ``extra_flags``: A/B variants of the kernel library (e.g. ``-DDML_PHASE_PROF``
    into ``lib/libdml_hip_phase.so``, loaded through ``DML_HIP_LIB``)."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")))
    os.makedirs(LIB, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result",
             "-I", os.path.join(CSRC, "kernels"), *extra_flags]
    # staleness by CONTENT (sources + headers + flags), never by mtime: the .so files are
    # git-ignored but travel with the tree to the GPU box, where every file has a fresh
    # mtime -- an mtime test there could keep a library that does not match the sources
    with _BuildLock():
        if force or _stale_by_hash(out, srcs + hdrs, flags):
            _build_hip_locked(out, srcs, hdrs, flags, force)
    return out


def _build_hip_locked(out, srcs, hdrs, flags, force) -> None:
    # one hipcc per translation unit, in parallel (forest.hip alone is most of the
    # build), then one link; a unit whose own content hash is unchanged keeps its object
    from concurrent.futures import ThreadPoolExecutor

    objdir = os.path.join(LIB, "obj", os.path.basename(out)[:-3])
    os.makedirs(objdir, exist_ok=True)
    objs = [os.path.join(objdir, os.path.basename(s)[:-4] + ".o") for s in srcs]

    def compile_one(so):
        src, obj = so
        if force or _stale_by_hash(obj, [src] + hdrs, flags):
            _run([_hipcc(), *flags, "-c", src, "-o", obj])
            _stamp(obj, [src] + hdrs, flags)

    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        list(ex.map(compile_one, zip(srcs, objs)))
    tmp = _tmp(out)
    _run([_hipcc(), f"--offload-arch={ARCH}", "-shared", *objs, "-o", tmp])
    os.replace(tmp, out)
    _stamp(out, srcs + hdrs, flags)


def build_cpu(force: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    deps = srcs + sorted(glob.glob(os.path.join(CSRC, "runtime", "*.h")) + glob.glob(os.path.join(CSRC, "kernels", "*.h")))
    os.makedirs(LIB, exist_ok=True)
    cxx = os.environ.get("CXX", shutil.which("g++") or "c++")
    flags = [cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-fopenmp", "-ffp-contract=off"]
    with _BuildLock():
        if force or _stale_by_hash(CPU_LIB, deps, flags):
            tmp = _tmp(CPU_LIB)
            _run([*flags, "-I", os.path.join(CSRC, "kernels"), *srcs, "-o", tmp])
            os.replace(tmp, CPU_LIB)
            _stamp(CPU_LIB, deps, flags)
    return CPU_LIB


SAN_EXE = os.path.join(LIB, "host_selftest_asan")


def build_sanitized(force: bool = False) -> str:
    """Host runtime + ``csrc/tests/host_selftest.cpp`` with AddressSanitizer and
    UndefinedBehaviorSanitizer (host code only — GPU sanitizers are not used on MI355X
    here).  Any report aborts the executable (``-fno-sanitize-recover=all``)."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))) + [os.path.join(CSRC, "tests", "host_selftest.cpp")]
    deps = srcs + glob.glob(os.path.join(CSRC, "kernels", "*.h"))
    os.makedirs(LIB, exist_ok=True)
    cxx = os.environ.get("CXX", shutil.which("g++") or "c++")
    flags = [cxx, "-O1", "-g", "-std=c++17", "-fopenmp", "-ffp-contract=off", "-fsanitize=address,undefined",
             "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]
    with _BuildLock():
        if force or _stale_by_hash(SAN_EXE, deps, flags):
            tmp = _tmp(SAN_EXE)
            _run([*flags, "-I", os.path.join(CSRC, "kernels"), *srcs, "-o", tmp])
            os.replace(tmp, SAN_EXE)
            _stamp(SAN_EXE, deps, flags)
    return SAN_EXE


def build_all(force: bool = False) -> tuple[str, str]:
    return build_cpu(force), build_hip(force)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--cpu-only", action="store_true")
    ap.add_argument("--sanitize", action="store_true", help="also build the ASan/UBSan host self-test")
    ap.add_argument("--variant", help="build an A/B kernel library lib/libdml_hip_<variant>.so instead")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="preprocessor define for --variant")
    args = ap.parse_args()
    if args.variant:
        print(build_hip(True, os.path.join(LIB, f"libdml_hip_{args.variant}.so"), tuple("-D" + d for d in args.defines)))
        sys.exit(0)
    if args.sanitize:
        print(build_sanitized(args.force))
    print(build_cpu(args.force))
    if not args.cpu_only:
        print(build_hip(args.force))
