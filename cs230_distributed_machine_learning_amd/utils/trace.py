"""Tracing: roctx ranges + host-side phase timers.

The reference has no tracing beyond ad-hoc ``training_time`` / timestamp fields and a
psutil sampler (aws-prod/worker/worker.py:198-221, 314-316).  Here every
slice / fit batch / kernel phase opens a named range that

* is pushed to ``libroctx64`` (ROCm's marker API), so ``rocprofv3 --marker-trace``
  timelines show the framework phases around the kernels they launch, and
* accumulates host wall time per range name (``summary()``), which the bench scripts
  print as a phase breakdown.

``DML_TRACE=0`` disables both (the ranges then cost one attribute check);
``DML_TRACE_SYNC=1`` synchronises the device at every range exit so host timers include
the GPU work launched inside (debug attribution only: it serialises the pipeline).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading
import time
from typing import Dict, Optional, Tuple

_ENABLED = os.environ.get("DML_TRACE", "1") != "0"
_SYNC = os.environ.get("DML_TRACE_SYNC", "0") == "1"
_lib: Optional[ctypes.CDLL] = None
_lib_tried = False
_lock = threading.Lock()
_stats: Dict[str, Tuple[int, float]] = {}


def _roctx() -> Optional[ctypes.CDLL]:
    global _lib, _lib_tried
    if _lib_tried:
        return _lib
    _lib_tried = True
    for name in ("libroctx64.so", "libroctx64.so.4", os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"),
                                                                  "lib", "libroctx64.so")):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _lib = lib
            break
        except (OSError, AttributeError):
            continue
    return _lib


def enabled() -> bool:
    return _ENABLED


def set_enabled(on: bool) -> None:
    global _ENABLED
    _ENABLED = bool(on)


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    if not _ENABLED:
        yield
        return
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if _SYNC:
            import torch

            if torch.cuda.is_available() and torch.cuda.is_initialized():
                torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if lib is not None:
            lib.roctxRangePop()
        key = name.split(" ", 1)[0] if " " in name else name
        with _lock:
            c, s = _stats.get(key, (0, 0.0))
            _stats[key] = (c + 1, s + dt)


def mark(msg: str) -> None:
    if _ENABLED:
        lib = _roctx()
        if lib is not None:
            lib.roctxMarkA(msg.encode())


def summary(reset: bool = False) -> Dict[str, Dict[str, float]]:
    with _lock:
        out = {k: {"count": c, "seconds": round(s, 6)} for k, (c, s) in sorted(_stats.items(), key=lambda kv: -kv[1][1])}
        if reset:
            _stats.clear()
    return out


def roctx_available() -> bool:
    return _roctx() is not None
