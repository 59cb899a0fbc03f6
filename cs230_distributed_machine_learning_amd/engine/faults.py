"""Fault injection and bounded retries for worker slices.

The reference has no fault injection (only a commented-out 30-45 s sleep,
aws-prod/worker/worker.py:308-311) and never retries a failed task: a failed subtask is
reported once and the job hangs below 100 % (D5, master/task_handler.py:91).  Here:

* a slice whose device batch raises a transient error (OOM, injected fault) is retried
  up to ``Config.max_retries`` times on the same rank before its candidates are failed
  with the error (they then count as terminal and take ``error_score``); a sticky device
  fault (HIP error) is not retried in-process under the distributed runner: the worker
  exits and the dispatcher re-queues its slice on a survivor (parallel/runner.py);
* ``DML_INJECT_FAIL_RATE`` (0..1) makes a deterministic fraction of slice *attempts*
  raise ``InjectedFault`` — decided by a hash of (job seed, slice, attempt), so a test
  can predict exactly which attempts fail;
* ``DML_KILL_RANK_AFTER="<rank>:<k>"`` makes that rank hard-exit (``os._exit``) right
  after claiming its (k+1)-th slice, i.e. with claimed-but-unpublished work — what a
  crashed GPU process looks like to the controller, which must detect the silence and
  re-queue the slice to the survivors.
* ``DML_STOP_RANK_IN="<rank>:<collective>"`` (``load`` / ``scores`` side-group tasks, ``dp``
  a data-parallel epoch, right after its table scatter) makes that rank SIGSTOP
  itself on entering the named collective: a HUNG peer (its sockets stay open,
  unlike a dead one), which the survivors' collective timeouts must turn into a fallback;
  ``DML_FAIL_RANK_IN`` (same form) makes it raise there instead;
  ``DML_OOM_RANK_IN`` (same form, ``load``) makes it run out of memory allocating the
  load's receive buffers (every rank then gives that load up together).
"""
from __future__ import annotations

import os
import zlib
from dataclasses import dataclass
from typing import Optional, Tuple


class InjectedFault(RuntimeError):
    pass


class InjectedOOM(RuntimeError):
    """Stands in for ``torch.cuda.OutOfMemoryError`` on a CPU box (fault injection)."""


@dataclass(frozen=True)
class FaultPlan:
    fail_rate: float = 0.0
    kill_rank: Optional[int] = None
    kill_after: int = 0
    max_retries: int = 2

    @classmethod
    def from_env(cls) -> "FaultPlan":
        rate = float(os.environ.get("DML_INJECT_FAIL_RATE", "0") or 0.0)
        kill = os.environ.get("DML_KILL_RANK_AFTER", "")
        kr, ka = None, 0
        if kill:
            a, _, b = kill.partition(":")
            kr, ka = int(a), int(b or 0)
        retries = int(os.environ.get("DML_MAX_RETRIES", "2"))
        return cls(min(max(rate, 0.0), 1.0), kr, ka, max(0, retries))

    def should_fail(self, seed: int, slice_key: str, attempt: int) -> bool:
        if self.fail_rate <= 0.0:
            return False
        h = zlib.crc32(f"{seed}:{slice_key}:{attempt}".encode()) & 0xFFFFFFFF
        return h < self.fail_rate * 4294967296.0

    def kill_now(self, rank: int, slices_done: int) -> bool:
        return self.kill_rank is not None and rank == self.kill_rank and slices_done >= self.kill_after


_PLAN: Optional[FaultPlan] = None


def plan() -> FaultPlan:
    global _PLAN
    if _PLAN is None:
        _PLAN = FaultPlan.from_env()
    return _PLAN


def reset() -> None:
    """Re-read the environment (tests)."""
    global _PLAN
    _PLAN = None


def maybe_inject(seed: int, slice_key: str, attempt: int) -> None:
    if plan().should_fail(seed, slice_key, attempt):
        raise InjectedFault(f"injected fault (slice {slice_key}, attempt {attempt})")


def _rank_spec(var: str, rank: int, what: str) -> bool:
    spec = os.environ.get(var, "")
    if not spec:
        return False
    r, _, w = spec.partition(":")
    return int(r) == rank and w == what


def maybe_stop_in_collective(rank: int, what: str) -> None:
    """Fault injection on entering a side-group collective (``load`` / ``scores``):
    ``DML_STOP_RANK_IN`` hangs the rank (SIGSTOP), ``DML_FAIL_RANK_IN`` makes it raise before
    the collective (an OOM while its peers are already inside), ``DML_COLL_DELAY_S`` delays
    every rank (a long broadcast), ``DML_DELAY_RANK_IN`` one rank (a slow peer)."""
    delay = float(os.environ.get("DML_COLL_DELAY_S", "0") or 0.0)
    # DML_DELAY_RANK_IN="rank:kind:seconds": ONE slow (not hung) rank entering that collective
    slow = os.environ.get("DML_DELAY_RANK_IN", "")
    if slow:
        r, k, sec = slow.split(":")
        if int(r) == rank and k in (what, "*"):
            delay += float(sec)
    if delay > 0:
        import time

        time.sleep(delay)
    if _rank_spec("DML_FAIL_RANK_IN", rank, what):
        raise InjectedFault(f"injected {what} collective failure on rank {rank}")
    if _rank_spec("DML_STOP_RANK_IN", rank, what):
        import signal

        os.kill(os.getpid(), signal.SIGSTOP)


def maybe_oom_in_collective(rank: int, what: str) -> None:
    """``DML_OOM_RANK_IN="<rank>:<collective>"``: that rank runs out of memory allocating its
    receive buffers for the named side-group task (``load``)."""
    if _rank_spec("DML_OOM_RANK_IN", rank, what):
        raise InjectedOOM(f"injected out-of-memory allocating the {what} buffers on rank {rank}")


def maybe_delay_staging() -> None:
    """``DML_STAGE_DELAY_S``: every host staging takes that much longer (a large table)."""
    d = float(os.environ.get("DML_STAGE_DELAY_S", "0") or 0.0)
    if d > 0:
        import time

        time.sleep(d)


def maybe_kill(rank: int, slices_done: int) -> None:
    if plan().kill_now(rank, slices_done):
        os._exit(17)


def run_with_retries(fn, seed: int, slice_key: str, retries: Optional[int] = None,
                     reraise=None) -> Tuple[object, int, Optional[BaseException]]:
    """Call ``fn()`` with up to ``retries`` re-tries -> (value, attempts, last error).

    ``value`` is None when every attempt raised.  ``reraise(e) -> bool`` marks errors that
    must not be retried in this process (a sticky device fault): they propagate."""
    n = plan().max_retries if retries is None else retries
    last: Optional[BaseException] = None
    for attempt in range(n + 1):
        try:
            maybe_inject(seed, slice_key, attempt)
            return fn(), attempt + 1, None
        except (RuntimeError, OSError, MemoryError) as e:  # OOM / injected / transient: retry the batch
            if getattr(e, "abort_epoch", False):   # a row-sharded collective failed: never retried here
                raise
            if reraise is not None and reraise(e):
                raise
            last = e
            _release_device_memory()
        except Exception as e:  # deterministic (parameter / data) errors are not retried
            return None, attempt + 1, e
    return None, n + 1, last


def _release_device_memory() -> None:
    try:
        import torch

        if torch.cuda.is_available():
            torch.cuda.empty_cache()
    except Exception:
        pass
