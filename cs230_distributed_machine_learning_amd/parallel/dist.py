"""Process-group plumbing: one process per GPU, ``torch.distributed`` over RCCL/xGMI.

Replaces the reference's transport layer (Kafka topics tasks/train/result/metrics,
Redis, HTTP heartbeats) for the single-node design:
* collectives (dataset all-gather/broadcast, score all-reduce) go over RCCL — the
  ``nccl`` backend IS RCCL on ROCm — and ride the point-to-point xGMI links;
* small control traffic (job announcements, work-claim counters, heartbeats) goes
  through the rendezvous ``TCPStore`` (``store.add`` is an atomic counter).
On a CPU box the same code runs on ``gloo`` (tests use world_size 2).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"

    @property
    def is_dist(self) -> bool:
        """A process group exists (world > 1, or DML_FORCE_PG=1 at world 1): collectives run."""
        return self.backend != "none" and dist.is_initialized()

    @property
    def is_root(self) -> bool:
        return self.rank == 0


_INFO: Optional[DistInfo] = None
_GEN = 0   # communicator generation of the current default group (0 = the launch group)


def _failure_env() -> None:
    """RCCL failure handling: a collective that outlives its timeout (a peer
    rank died or hung mid-collective) must not take the service down with it.  Mode 2
    (CleanUpOnly) makes the watchdog abort the communicator WITHOUT tearing the process
    down, and blocking wait makes the timed-out collective raise in the thread that issued
    it -- the runner's collective thread / data-parallel epoch then reports the error and
    the dispatcher re-forms the group (parallel/runner.py).  Mode 1 (TearDown) would end
    every survivor, rank 0 (controller + gateway + store) included.  The monitor thread
    std::abort()s a process whose watchdog looks stuck (an abort that itself blocks): that
    is a teardown too."""
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")
    os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "1")
    os.environ.setdefault("TORCH_NCCL_ENABLE_MONITORING", "0")


def init(backend: Optional[str] = None, timeout_s: float = 1800.0, want_gpu: Optional[bool] = None) -> DistInfo:
    """Initialise from torchrun env vars (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*)."""
    global _INFO
    if _INFO is not None:
        return _INFO
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # multi-rank rehearsal on a one-GPU box: every rank shares device 0 and the
    # collectives go over gloo (RCCL refuses two ranks on one device)
    if os.environ.get("DML_SHARE_DEVICE") == "1":
        local = 0
    backend = backend or os.environ.get("DML_DIST_BACKEND") or None
    gpu = torch.cuda.is_available() if want_gpu is None else want_gpu
    if gpu:
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    be = "none"
    # DML_FORCE_PG=1: build the process group even for one rank, so the RCCL code path
    # (communicator setup, every collective the runner and bench use) runs on a one-GPU box
    force = os.environ.get("DML_FORCE_PG") == "1"
    if world > 1 or force:
        be = backend or ("nccl" if gpu else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29561")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        _failure_env()
        timeout_s = float(os.environ.get("DML_COLLECTIVE_TIMEOUT_S", timeout_s))
        kw = dict(backend=be, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    _INFO = DistInfo(rank, world, local, device, be)
    return _INFO


def info() -> DistInfo:
    return _INFO or DistInfo()


def generation() -> int:
    return _GEN


def regroup_timeout_s() -> float:
    """How long a communicator re-formation waits for every member (``DML_REGROUP_TIMEOUT_S``,
    default 60 s); also the per-collective timeout of the re-formed default group's setup."""
    return float(os.environ.get("DML_REGROUP_TIMEOUT_S", "60"))


class RegroupError(RuntimeError):
    """A communicator generation could not be formed (a member never arrived or failed)."""


def regroup(base_store, gen: int, rank: int, world: int, backend: str, device: torch.device,
            local_rank: int = 0, timeout_s: Optional[float] = None) -> DistInfo:
    """Leave the current process group (if any) and join communicator generation ``gen``:
    ``world`` members, this process at ``rank``, rendezvous under the store prefix
    ``gen<g>/`` of the service's control-plane store ``base_store`` -- the same TCPStore the
    launch group used, so survivors, respawned ranks and processes that joined later
    (which never had a process group) meet on equal terms.  The side and data-parallel
    communicators are rebuilt on the new group.  Every member calls this with the same
    ``gen``/``world``/``backend``; a member that is missing after ``timeout_s`` makes every
    other member raise ``RegroupError`` before any communicator is built (a presence
    rendezvous on the store precedes the process-group constructor, which would otherwise
    block for its full timeout).  On failure this process is left with NO process group."""
    global _INFO, _SIDE, _DP, _GEN
    from torch.distributed import PrefixStore

    timeout_s = regroup_timeout_s() if timeout_s is None else float(timeout_s)
    _SIDE = None
    _DP = None
    if dist.is_initialized():
        try:
            dist.destroy_process_group()
        except Exception:   # a communicator already aborted by its watchdog
            pass
    _INFO = DistInfo(rank, world, local_rank, device, "none")
    st = PrefixStore(f"gen{gen}", base_store)
    st.set(f"here/{rank}", "1")
    try:
        st.wait([f"here/{r}" for r in range(world)], datetime.timedelta(seconds=timeout_s))
    except Exception as e:
        raise RegroupError(f"generation {gen}: not every member arrived within {timeout_s:.0f}s") from e
    _failure_env()
    coll_timeout = float(os.environ.get("DML_COLLECTIVE_TIMEOUT_S", "1800"))
    kw = dict(backend=backend, store=PrefixStore("pg", st), rank=rank, world_size=world,
              timeout=datetime.timedelta(seconds=coll_timeout))
    if backend == "nccl":
        kw["device_id"] = device
    try:
        dist.init_process_group(**kw)
    except Exception as e:
        raise RegroupError(f"generation {gen}: process group init failed: {e}") from e
    _INFO = DistInfo(rank, world, local_rank, device, backend)
    _GEN = gen
    try:
        side_group()
        dp_group()
    except Exception as e:
        _SIDE = _DP = None
        try:
            dist.destroy_process_group()
        except Exception:
            pass
        _INFO = DistInfo(rank, world, local_rank, device, "none")
        raise RegroupError(f"generation {gen}: side / data-parallel communicators failed: {e}") from e
    # every member is through: the presence keys can go (rank 0 only, after a barrier)
    barrier()
    if rank == 0:
        for r in range(world):
            st.delete_key(f"here/{r}")
    return _INFO


def leave_group() -> None:
    """Drop this process's communicators (a member that failed a re-formation, or that left
    the group): ``info().is_dist`` is False until the next ``regroup``."""
    global _INFO, _SIDE, _DP
    _SIDE = _DP = None
    if dist.is_initialized():
        try:
            dist.destroy_process_group()
        except Exception:
            pass
    if _INFO is not None:
        _INFO = DistInfo(_INFO.rank, _INFO.world, _INFO.local_rank, _INFO.device, "none")


_SIDE = None


def side_group():
    """A second communicator over every rank (created collectively, at WorkerCore setup):
    the cluster runner's collective thread broadcasts new datasets and all-gathers job
    scores on it WHILE the worker threads run slices on the default stream -- no rank is
    drained for a collective (parallel/runner.py).  None when not distributed."""
    global _SIDE
    if not info().is_dist:
        return None
    if _SIDE is None:
        # a SHORT timeout: a side collective stuck on a dead or hung peer raises here after
        # side_timeout_s() instead of the default group's long one, and the runner falls back
        # to host staging / store copies (parallel/runner.py _break_group)
        _SIDE = dist.new_group(ranks=list(range(info().world)), backend=info().backend,
                               timeout=datetime.timedelta(seconds=side_timeout_s()))
    return _SIDE


_DP = None


class CollectiveAborted(RuntimeError):
    """Every rank of a side-group task gave it up TOGETHER before any large collective was
    entered (a rank could not allocate its buffers -- OOM -- or rank 0 could not prepare the
    table): the communicator is intact, only this task falls back (host staging)."""

    consistent = True


def vote_all_ok(ok: bool, group=None) -> bool:
    """True when every rank of ``group`` passed ``ok`` (one tiny MIN all-reduce).  Used before
    a large collective so a rank that cannot take part (OOM on its receive buffer) makes
    every rank skip the collective, instead of leaving its peers stuck inside it."""
    if not info().is_dist:
        return ok
    dev = info().device if info().backend == "nccl" else torch.device("cpu")
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


class CollectiveError(RuntimeError):
    """A collective of a row-sharded (data-parallel) epoch failed or timed out: a peer died,
    hung, or ran out of memory.  The epoch's communicator is unusable from here on, so the
    error aborts the whole epoch (never a per-batch retry, never "failed candidates") and the
    dispatcher re-runs the job task-parallel on the survivors (parallel/runner.py)."""

    abort_epoch = True


def dp_group():
    """The communicator of data-parallel epochs (created collectively at WorkerCore setup,
    after ``side_group``): its own SHORT per-collective timeout, so a rank that dies or hangs
    mid-epoch costs the survivors ``dp_timeout_s()`` -- not the default group's 30 minutes --
    before their collective raises.  None when not distributed."""
    global _DP
    if not info().is_dist:
        return None
    if _DP is None:
        _DP = dist.new_group(ranks=list(range(info().world)), backend=info().backend,
                             timeout=datetime.timedelta(seconds=dp_timeout_s()))
    return _DP


def dp_timeout_s() -> float:
    """Per-collective timeout of the data-parallel communicator (``DML_DP_TIMEOUT_S``,
    default 300 s: covers rank 0 parsing a large table while its peers wait in the scatter;
    every later collective of an epoch is a sub-second all-reduce between equal shards)."""
    return float(os.environ.get("DML_DP_TIMEOUT_S", "300"))


def side_timeout_s() -> float:
    """Per-collective timeout of the side communicator (``DML_SIDE_TIMEOUT_S``, default 120 s:
    a 40 GB table broadcast over xGMI takes well under that)."""
    return float(os.environ.get("DML_SIDE_TIMEOUT_S", "120"))


def barrier(group=None) -> None:
    if info().is_dist:
        if info().backend == "nccl":
            dist.barrier(group=group, device_ids=[info().local_rank])
        else:
            dist.barrier(group=group)


def broadcast(t: torch.Tensor, src: int = 0, group=None) -> torch.Tensor:
    if info().is_dist:
        dist.broadcast(t, src=src, group=group)
    return t


def all_gather_rows(shard: torch.Tensor, group=None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Concatenate equal-size row shards of every rank (rank order) on every rank (into
    ``out`` when given: a caller that pre-allocates can vote on the allocation first)."""
    inf = info()
    if not inf.is_dist:
        return shard
    shard = shard.contiguous()
    if out is None:
        out = torch.empty((shard.shape[0] * inf.world, *shard.shape[1:]), dtype=shard.dtype, device=shard.device)
    if inf.backend == "nccl":
        dist.all_gather_into_tensor(out, shard, group=group)
    else:
        parts = list(out.chunk(inf.world, 0))
        dist.all_gather(parts, shard, group=group)
    return out


def all_reduce_sum(t: torch.Tensor) -> torch.Tensor:
    if info().is_dist:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def all_reduce_max(t: torch.Tensor) -> torch.Tensor:
    if info().is_dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t


def gather_objects(obj) -> List:
    inf = info()
    if not inf.is_dist:
        return [obj]
    out: List = [None] * inf.world
    dist.all_gather_object(out, obj)
    return out


def store():
    """The default group's TCPStore (None when not distributed)."""
    if not info().is_dist:
        return None
    from torch.distributed.distributed_c10d import _get_default_store

    return _get_default_store()


def service_store():
    """The runner's control-plane store: the rendezvous TCPStore under the fixed prefix
    ``dml`` -- the same view whether a process is a member of the process group (walks
    past the group's own key prefixes) or joined later with just the host and port
    (``parallel/runner.py join_cluster``)."""
    from torch.distributed import PrefixStore

    st = store()
    if st is None:
        return None
    raw = st
    while getattr(raw, "underlying_store", None) is not None:
        raw = raw.underlying_store
    return PrefixStore("dml", raw)


def service_client(timeout_s: float = 300.0):
    """A NEW connection to the control-plane store (same ``dml`` view as service_store):
    a thread that blocks in ``TCPStore.wait`` on its own client never holds up the
    threads sharing the main one (parallel/runner.py)."""
    import datetime

    from torch.distributed import PrefixStore, TCPStore

    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "29500"))
    raw = TCPStore(host, port, is_master=False, timeout=datetime.timedelta(seconds=timeout_s))
    return PrefixStore("dml", raw)


def destroy() -> None:
    global _INFO, _SIDE, _DP, _GEN
    _SIDE = None
    _DP = None
    _GEN = 0
    if dist.is_initialized():
        dist.destroy_process_group()
    _INFO = None
