"""Distributed job runner: one rank per GPU; rank 0 = controller + gateway + dispatcher + worker.

Replaces the reference's scheduler/worker tiers and their Kafka/HTTP plumbing
(aws-prod/scheduler/scheduler_service.py:173-191 placement, :197-351 ingress/status
loops, :205-247 heartbeat monitor + requeue; scheduler.py:105-139 subscribe/unsubscribe;
worker/worker.py:156-286 consume loop):

jobs               every submitted job is admitted at once and cut into LPT slices
                   (most expensive first); the cluster runs the slices of ALL active jobs
                   concurrently, like the reference scheduler interleaving every job's
                   tasks across every worker
dispatch           rank 0's dispatcher hands each idle worker its next slice through the
                   rendezvous TCPStore (``asg/<worker>/<k>`` -> ``res/<worker>/<k>``); the
                   slice comes from the active job of the session that has used the least
                   node time so far (slice-level fair share, the same policy as the local
                   runner), so a one-candidate job overtakes a running 256-candidate search
dataset            once per dataset per worker.  While the whole process group is alive every
                   rank receives the table by ONE RCCL broadcast over xGMI (parallel/data.py)
                   issued by the rank's *collective thread* on a second communicator
                   (dist.side_group) and its own HIP stream: the worker threads keep running
                   slices of resident datasets meanwhile -- nothing is drained for a load.
                   Once a rank has died (the default group can no longer run collectives) or
                   for a worker that joined after launch, rank 0 stages the table in a host
                   file and each worker copies it to its own GPU over its own PCIe link
results            every rank keeps the score rows of the candidates it ran; when a job's last
                   slice lands, the collective threads all-gather them over RCCL (side group)
                   (all_gather_into_tensor of a [candidates, width] float64 tensor) and rank
                   0 builds the job's final records (J5) from that tensor -- the reference's
                   Kafka ``result`` channel (worker.py:247-254 -> task_handler.py:18-50).  The
                   per-slice store message is the control / progress copy (status and SSE
                   stream as slices land; the fallback once the group is broken or for a
                   joined worker, whose rows no collective can reach).  Rank 0 holds each
                   job's last slice until the best candidate is refit, so "completed"
                   always carries the model
liveness           every worker refreshes ``hb/<worker>``; a worker silent for
                   ``dead_after_s`` is declared dead, its in-flight slice goes back to the
                   front of its job's queue and the survivors finish the job.  A slice that
                   hits a device fault makes its worker exit (a poisoned HIP context cannot
                   retry in-process); the dispatcher re-queues it the same way
membership         processes outside the launch world can join at any time
                   (``join_cluster``; /subscribe): they get a worker id, heartbeat, and
                   receive slices with host-staged datasets; they leave by unsubscribing or
                   by dying (reference scheduler.py:105-139 elastic join/leave)
data parallel      row-sharded jobs (parallel/data_parallel.py) run as an exclusive epoch on
                   every rank of the process group, only while it is whole; otherwise they
                   fall back to task-parallel slices
"""
from __future__ import annotations

import collections
import json
import os
import queue
import tempfile
import threading
import time
import traceback
import zlib
from dataclasses import dataclass, field
from typing import Any, Deque, Dict, List, Optional, Set

import numpy as np
import torch

from ..engine import faults
from ..engine.jobs import Job, json_safe
from ..engine.service import (Controller, Runner, attach_model, candidate_costs, job_plan, job_seed, pick_refit,
                              plan_slices, presize_for_job, publish_results, refit_model, run_slice,
                              should_recut)
from ..models.base import family_of, is_classifier
from ..utils.log import get_logger
from . import data as pdata
from . import dist

log = get_logger("dml.runner")

HB_PERIOD_S = 1.0
POLL_S = 0.003
MAX_WORKERS = 4096


class LockedStore:
    """Thread-safe view of a TCPStore client (rank 0's dispatcher, its worker thread and
    the heartbeat share one client).  ``wait`` blocks server-side (``TCPStore.wait``) on a
    PRIVATE client when one is given (``waiter``: no lock held, no polling), else polls
    ``check``.  ``ops`` counts the store operations this view issued (control-plane load,
    profiles/r3_cluster_8rank_gloo.log)."""

    def __init__(self, store, waiter=None):
        self._s = store
        self._lock = threading.Lock()
        self._waiter = waiter
        self.ops = 0

    def add(self, k, v):
        with self._lock:
            self.ops += 1
            return self._s.add(k, v)

    def set(self, k, v):
        with self._lock:
            self.ops += 1
            return self._s.set(k, v)

    def get(self, k):
        with self._lock:
            self.ops += 1
            return self._s.get(k)

    def check(self, ks):
        with self._lock:
            self.ops += 1
            return self._s.check(ks)

    def delete_key(self, k):
        with self._lock:
            self.ops += 1
            try:
                return self._s.delete_key(k)
            except Exception:
                return False

    def wait(self, ks, timeout=None, poll_s: float = 0.002):
        if self._waiter is not None:
            import datetime

            t = 24 * 3600.0 if timeout is None else max(0.001, float(timeout))
            self.ops += 1
            try:
                self._waiter.wait(ks, datetime.timedelta(seconds=t))
            except Exception as e:   # DistStoreError: timeout, or the store is gone
                if "timeout" in str(e).lower() or "timed out" in str(e).lower():
                    raise TimeoutError(ks) from e
                raise
            return
        t0 = time.time()
        while True:
            if self.check(ks):
                return
            if timeout is not None and time.time() - t0 > timeout:
                raise TimeoutError(ks)
            time.sleep(poll_s)


SCORE_HEAD = 4   # score row: [ok, mean_cv_score, std_cv_score, n_cv, cv_0 .. cv_{n_cv-1}]


def score_width(plan: Dict[str, Any]) -> int:
    """Columns of a job's score rows: the head plus one per CV fold (``cv`` is the user's
    integer, reference aws-prod/master/task_handler.py:183,203 -- never truncated)."""
    try:
        cv = int(plan.get("cv", 5))
    except (TypeError, ValueError):
        cv = 5
    return SCORE_HEAD + max(1, cv)


def score_row(ok: bool, result: Dict[str, Any], width: int) -> np.ndarray:
    """A candidate's numeric result as one float64 row (NaN padded) for the scores epoch."""
    row = np.full(width, np.nan, dtype=np.float64)
    row[0] = 1.0 if ok else 0.0
    if ok:
        cvs = list(result.get("cv_scores") or [])[:width - SCORE_HEAD]
        row[1] = float(result.get("mean_cv_score", np.nan))
        row[2] = float(result.get("std_cv_score", np.nan))
        row[3] = len(cvs)
        row[SCORE_HEAD:SCORE_HEAD + len(cvs)] = [np.nan if v is None else float(v) for v in cvs]
    return row


class _Res:
    """Lightweight CandidateResult rebuilt from store JSON."""

    def __init__(self, d: Dict[str, Any]):
        self.candidate = int(d["candidate"])
        self.ok = bool(d["ok"])
        self.result = d.get("result") or {}
        self.error = d.get("error")
        self.fit_seconds = float(d.get("fit_seconds", 0.0))


def _enc_results(results, metrics) -> List[Dict[str, Any]]:
    out = []
    for r in results:
        out.append({"candidate": r.candidate, "ok": r.ok, "result": json_safe(r.result), "error": r.error,
                    "fit_seconds": r.fit_seconds, "metrics": json_safe(metrics.get(r.candidate))})
    return out


class _Heartbeat:
    def __init__(self, store, wid: int):
        self.store, self.wid = store, wid
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._loop, daemon=True, name=f"dml-hb-{wid}")
        self._t.start()

    def _loop(self):
        while True:
            try:
                self.store.set(f"hb/{self.wid}", str(time.time()))
            except Exception:
                return
            if self._stop.wait(HB_PERIOD_S):
                return

    def stop(self):
        self._stop.set()


_DEVICE_FAULT_MARKERS = ("HIP error", "hipError", "CUDA error", "device-side assert", "HSA_STATUS",
                         "illegal memory access", "GPU fault", "unspecified launch failure", "memory access fault")


def is_device_fault(e: BaseException) -> bool:
    """A sticky device fault poisons the process's HIP context: nothing more can run here."""
    if isinstance(e, faults.InjectedFault) or isinstance(e, torch.cuda.OutOfMemoryError):
        return False
    msg = f"{type(e).__name__}: {e}"
    return isinstance(e, RuntimeError) and any(m in msg for m in _DEVICE_FAULT_MARKERS)


def dataset_key(registry, dataset_id: str, plan: Dict[str, Any]) -> str:
    path = registry.find_file(dataset_id)
    mt = os.path.getmtime(path) if path and os.path.exists(path) else 0
    return f"{path}:{mt}:{plan['feature_columns']}:{plan['target_column']}:{is_classifier(plan['model_type'])}"


def _needs_bins(plan) -> bool:
    return plan["model_type"].startswith("RandomForest") or plan["model_type"].startswith("GradientBoosting")


class WorkerCore:
    """What a worker does with an assignment (every rank; rank 0 also has the controller)."""

    def __init__(self, device: torch.device, wid: Optional[int] = None, store=None, in_group: bool = True):
        self.inf = dist.info()
        self.wid = self.inf.rank if wid is None else wid
        if store is None:   # the shared client + a private one this worker blocks on
            store = LockedStore(dist.service_store(), waiter=_private_client())
        self.store = store
        self.device = device
        self.in_group = in_group
        self.cache: "collections.OrderedDict[str, Any]" = collections.OrderedDict()
        self.msgs: Dict[int, Dict[str, Any]] = {}
        self.presized: Set[int] = set()
        self.slices_done = 0
        # scores epoch: this rank's score rows per job (seq -> candidate -> row) until the
        # job's all-gather; rank 0's merged [candidates, width + 1] table per job after it
        self.score_rows: Dict[int, Dict[int, np.ndarray]] = {}
        self.gathered: Dict[int, Any] = {}
        self.intervals: List[tuple] = []      # (kind, wall start, wall end) of collective work
        self.cache_lock = threading.RLock()   # the worker and the collective thread share the cache
        # the side communicator (collective with every rank: built here, by every in-group rank)
        self.side = dist.side_group() if (in_group and self.inf.is_dist) else None
        self.stage_dir: Optional[str] = None    # rank 0: the dispatcher's host staging directory
        self.load_h2d_s: List[float] = []       # this rank's H2D seconds per collective load
        # the data-parallel communicator (short timeout; created collectively right after the
        # side group, in the same order on every in-group rank)
        self.dp = dist.dp_group() if (in_group and self.inf.is_dist) else None
        self._coll_thread: Optional[threading.Thread] = None
        self.gen = 0                            # communicator generation this rank belongs to

    # ---- communicator generations -------------------------------------------------------
    def start_collective_thread(self, ctl: Optional[Controller], start: int = 0) -> None:
        if self.side is None:
            return
        t = threading.Thread(target=collective_loop, args=(self, ctl, start), daemon=True,
                             name=f"dml-coll-{self.wid}-g{self.gen}")
        self._coll_thread = t
        t.start()

    def regroup(self, a: Dict[str, Any], ctl: Optional[Controller]) -> Dict[str, Any]:
        """Join communicator generation ``a['gen']`` (dispatcher's regroup epoch): stop this
        rank's collective thread (the dispatcher posted a stop at the end of the task
        stream), leave the old process group, rendezvous with the other members on the
        control-plane store and build the new default / side / data-parallel communicators
        (parallel/dist.py regroup), then restart the collective thread at ``coll_base``.
        Survivors, respawned ranks and processes that joined later all become members."""
        t0 = time.perf_counter()
        old = self._coll_thread
        if old is not None and old.is_alive():
            old.join(timeout=dist.side_timeout_s() + 30.0)
            if old.is_alive():
                raise dist.RegroupError("the collective thread is still inside an old-generation collective")
        self._coll_thread = None
        members = [int(m) for m in a["members"]]
        rank = members.index(self.wid)
        dev = self.device
        local = dev.index if (dev.type == "cuda" and dev.index is not None) else 0
        self.side = self.dp = None
        self.in_group = False
        try:
            dist.regroup(self.store._s, int(a["gen"]), rank, len(members), a["backend"], dev, local_rank=local)
        except Exception:
            dist.leave_group()
            self.inf = dist.info()
            raise
        self.inf = dist.info()
        self.gen = int(a["gen"])
        self.in_group = True
        self.side = dist.side_group()
        self.dp = dist.dp_group()
        self.start_collective_thread(ctl, int(a["coll_base"]))
        return {"gen": self.gen, "rank": rank, "world": len(members), "wall": time.perf_counter() - t0}

    # ---- job messages and datasets ------------------------------------------------------
    def job_msg(self, seq: int) -> Dict[str, Any]:
        m = self.msgs.get(seq)
        if m is None:
            m = json.loads(self.store.get(f"job/{seq}"))
            m["_seq"] = seq
            self.msgs[seq] = m
            while len(self.msgs) > 64:
                self.msgs.pop(next(iter(self.msgs)))
        return m

    def _keep(self, key: str, dd) -> None:
        with self.cache_lock:
            self.cache[key] = dd
            self.cache.move_to_end(key)
            while len(self.cache) > 4:
                self.cache.popitem(last=False)

    def cache_keys(self) -> List[str]:
        with self.cache_lock:
            return list(self.cache.keys())

    def dataset(self, msg: Dict[str, Any], ctl: Optional[Controller] = None):
        """The job's resident table; loaded from the host-staged file when absent."""
        from ..data.device import DeviceData

        key = msg["dataset_key"]
        with self.cache_lock:
            dd = self.cache.get(key)
            if dd is not None:
                self.cache.move_to_end(key)
                return dd
        path = msg.get("staged")
        if not path and "_seq" in msg:   # cached before the dispatcher host-staged the table
            fresh = json.loads(self.store.get(f"job/{msg['_seq']}"))
            fresh["_seq"] = msg["_seq"]
            self.msgs[msg["_seq"]] = fresh
            path = fresh.get("staged")
        if not path:
            raise RuntimeError(f"dataset {msg['dataset_id']!r} is not resident on worker {self.wid} and not staged")
        X, y = pdata.load_staged(path, self.device)
        dd = DeviceData(X, y, is_classifier(msg["plan"]["model_type"]), self.device, name=msg["dataset_id"])
        self._keep(key, dd)
        return dd

    def load_collective(self, msg: Dict[str, Any], ctl: Optional[Controller], group=None, tag: str = ""):
        """Every rank receives the table by one broadcast (RCCL on GPU); on the side group
        (``group``, key suffix ``tag``) when the collective thread runs it."""
        from ..data.device import DeviceData

        plan = msg["plan"]
        clf = is_classifier(plan["model_type"])
        X = y = None
        mode_key = "dataset/mode" + tag
        if self.inf.rank == 0:
            try:
                ds = ctl.registry.load(msg["dataset_id"], plan["feature_columns"], plan["target_column"])
                X, y = ds.X, ds.y
                binned = ctl is not None and _binned_only_table(ctl, plan, X, self.device)
                mode = "binned" if binned else "full"
                if not binned and self.inf.world > 1 and self.stage_dir and X.nbytes >= shard_load_min_bytes():
                    # large table: staged once on the host, every rank copies its own 1/N row
                    # block over its own PCIe link, one all-gather over xGMI completes it
                    path = pdata.ensure_staged(lambda: (X, y), staged_path(self.stage_dir, msg["dataset_key"]))
                    mode = "sharded:" + path
            except Exception as e:   # every rank gives the load up together: no collective entered
                self.store_raw().set(mode_key, f"error:{type(e).__name__}: {e}")
                raise dist.CollectiveAborted(f"rank 0 could not prepare {msg['dataset_id']!r}: {e}") from e
            self.store_raw().set(mode_key, mode)
        else:
            # rank 0 parses (and, for a large table, host-stages) before it publishes the mode:
            # that is not a collective, so it is bounded by the load-preparation deadline, not
            # by the side timeout (a 1 GB+ CSV parse can outlast the latter); a rank 0 that
            # fails publishes an error mode instead
            import datetime

            self.store_raw().wait([mode_key], datetime.timedelta(seconds=load_prep_timeout_s()))
            mode = self.store_raw().get(mode_key).decode()
            if mode.startswith("error:"):
                raise dist.CollectiveAborted(f"rank 0 could not prepare {msg['dataset_id']!r}: {mode[6:]}")
            binned = mode == "binned"
        if mode.startswith("sharded:"):
            Xd, y_host, h2d = pdata.sharded_load(mode[len("sharded:"):], self.device, group=group)
            self.load_h2d_s.append(h2d)
            dd = DeviceData(Xd, y_host, clf, self.device, name=msg["dataset_id"])
            if _needs_bins(plan):
                pdata.share_bins(dd, group=group)
        elif binned:   # tree job on a table too large for HBM as float32: bins only
            dd = pdata.broadcast_binned(X, y, clf, self.device, name=msg["dataset_id"], group=group, tag=tag)
        else:
            Xd, y_host = pdata.broadcast_table(X, y, self.device, group=group, tag=tag)
            dd = DeviceData(Xd, y_host, clf, self.device, name=msg["dataset_id"])
            if _needs_bins(plan):
                pdata.share_bins(dd, group=group)
        dist.barrier(group=group)
        if self.inf.rank == 0:
            self.store_raw().delete_key(mode_key)
            if mode.startswith("sharded:"):   # the transient host copy, unless a staged job reads it
                pdata.release_staged(mode[len("sharded:"):])
        self._keep(msg["dataset_key"], dd)
        return dd

    @staticmethod
    def store_raw():
        return dist.store()

    # ---- assignments ----------------------------------------------------------------------
    def execute(self, a: Dict[str, Any], ctl: Optional[Controller]) -> Dict[str, Any]:
        kind = a["kind"]
        if kind == "slice":
            return self._slice(a, ctl)
        if kind == "load":
            msg = self.job_msg(a["seq"])
            t0 = time.perf_counter()
            self.load_collective(msg, ctl)
            return {"loaded": msg["dataset_key"], "wall": time.perf_counter() - t0, "cache": self.cache_keys()}
        if kind == "dp":
            return self._dp(a, ctl)
        if kind == "refit":
            return self._refit(a, ctl)
        if kind == "regroup":
            return self.regroup(a, ctl)
        if kind == "scores":
            return self._scores(a)
        raise ValueError(f"unknown assignment kind {kind!r}")

    def collective(self, a: Dict[str, Any], ctl: Optional[Controller], stream=None) -> Dict[str, Any]:
        """A task of the collective thread (side group, own stream): a dataset broadcast or
        a job's scores all-gather.  Every in-group rank runs the tasks in the same order."""
        t0 = time.perf_counter()
        tw0 = time.time()
        faults.maybe_stop_in_collective(self.wid, a["kind"])   # fault injection (tests)
        ctx = torch.cuda.stream(stream) if stream is not None else _null_ctx()
        with ctx:
            if a["kind"] == "load":
                msg = self.job_msg(a["seq"])
                self.load_collective(msg, ctl, group=self.side, tag=f"/c{a['i']}")
                out = {"loaded": msg["dataset_key"], "cache": self.cache_keys()}
            elif a["kind"] == "scores":
                out = self._scores(a, group=self.side)
            else:
                raise ValueError(f"unknown collective task {a['kind']!r}")
            if stream is not None:
                stream.synchronize()   # the table is complete before any slice may use it
        out["wall"] = time.perf_counter() - t0
        self.note_interval("side:" + a["kind"], tw0)
        return out

    def note_interval(self, kind: str, t0: float) -> None:
        """Wall-clock span of a collective task on this rank (tests check that side-group
        tasks and data-parallel epochs never overlap)."""
        self.intervals.append((kind, t0, time.time()))
        if len(self.intervals) > 4096:
            del self.intervals[:2048]

    def _scores(self, a, group=None) -> Dict[str, Any]:
        """Scores epoch of one job (every rank of the group): each rank contributes the score
        rows of the candidates it ran, ONE all_gather_into_tensor (RCCL over xGMI; gloo on
        CPU) assembles them, rank 0 keeps the merged table for the dispatcher."""
        seq, n, W = int(a["seq"]), int(a["n"]), int(a["width"])
        mine = self.score_rows.pop(seq, {})
        dev = self.inf.device if self.inf.is_dist else self.device
        t = torch.full((n, W + 1), float("nan"), dtype=torch.float64)
        t[:, W] = 0.0
        for c, row in mine.items():
            if 0 <= c < n:
                t[c, :W] = torch.from_numpy(row[:W])
                t[c, W] = 1.0
        allt = dist.all_gather_rows(t.to(dev), group=group).cpu().numpy().reshape(-1, n, W + 1)
        if self.inf.rank == 0:
            merged = np.full((n, W + 1), np.nan)
            merged[:, W] = 0.0
            for r in range(allt.shape[0]):          # a re-run slice: the first rank's row wins
                take = (allt[r, :, W] > 0) & (merged[:, W] == 0)
                merged[take] = allt[r, take]
            self.gathered[seq] = (merged, self.inf.backend)
        return {"scores": seq, "rows": len(mine), "backend": self.inf.backend}

    def _slice(self, a, ctl) -> Dict[str, Any]:
        msg = self.job_msg(a["seq"])
        faults.maybe_kill(self.wid, self.slices_done)   # fault injection: die holding an assigned slice
        t_load = time.perf_counter()
        dd = self.dataset(msg, ctl)
        if a["seq"] not in self.presized:   # job setup on this worker: size the device arena once
            self.presized.add(a["seq"])
            presize_for_job(msg["plan"], msg["params"], dd, msg["slices"])
        load_s = time.perf_counter() - t_load
        results, metrics, wall = run_slice(msg["plan"], msg["params"], msg["subtask_ids"], dd, a["ids"],
                                           f"rank{self.wid}", str(self.device), seed=msg["seed"],
                                           keep_models=msg.get("keep_models", "none"),
                                           models_root=msg.get("models_root"), fault_exit=True)
        self.slices_done += 1
        if self.in_group:   # kept for the job's scores epoch (parallel/runner.py header)
            rows = self.score_rows.setdefault(a["seq"], {})
            width = score_width(msg["plan"])
            for r in results:
                rows[r.candidate] = score_row(r.ok, r.result or {}, width)
        return {"results": _enc_results(results, metrics), "wall": wall, "load_s": load_s,
                "cache": self.cache_keys()}

    def _dp(self, a, ctl) -> Dict[str, Any]:
        """Data-parallel job on the whole process group: every rank runs every slice in
        order on its row shard (the fits' reductions are collectives), then all ranks
        refit the winner together; rank 0 decides the winner and keeps the model."""
        seq = a["seq"]
        msg = self.job_msg(seq)
        plan = msg["plan"]
        tw0 = time.time()
        try:
            return self._dp_run(seq, msg, plan, ctl)
        finally:
            self.note_interval("dp", tw0)

    def _dp_run(self, seq, msg, plan, ctl) -> Dict[str, Any]:
        from .data_parallel import RowShard, scatter_table

        X = y = None
        if self.inf.rank == 0:
            ds = ctl.registry.load(msg["dataset_id"], plan["feature_columns"], plan["target_column"])
            X, y = ds.X, ds.y
        Xs, y_glob, r0 = scatter_table(X, y, self.device, group=self.dp)
        dd = RowShard(Xs, y_glob, r0, is_classifier(plan["model_type"]), self.device, name=msg["dataset_id"],
                      group=self.dp)
        faults.maybe_stop_in_collective(self.wid, "dp")   # fault injection: a rank hangs mid-epoch
        out: List[Dict[str, Any]] = []
        results_all = []
        for ids in msg["slices"]:
            results, metrics, wall = run_slice(plan, msg["params"], msg["subtask_ids"], dd, ids, "data-parallel",
                                               str(self.device), seed=msg["seed"], retries=0)
            results_all.extend(results)
            out.append({"results": _enc_results(results, metrics), "wall": wall})
        # the winner is chosen by rank 0 (it owns the job table) and announced to every rank
        if self.inf.rank == 0:
            job = ctl.table.get(msg["session_id"], msg["job_id"])
            best = pick_refit(ctl, job, plan, results_all)
            self.store.set(f"job/{seq}/refit", str(best if best is not None else -1))
        else:
            try:
                self.store.wait([f"job/{seq}/refit"], timeout=dist.dp_timeout_s())
            except TimeoutError as e:   # rank 0 left the epoch (its collective failed first)
                raise dist.CollectiveError(f"no refit decision from rank 0 within {dist.dp_timeout_s():.0f}s") from e
        best_i = int(self.store.get(f"job/{seq}/refit"))
        model_path = None
        if best_i >= 0:
            model = refit_model(plan, msg["params"][best_i], dd)
            if self.inf.rank == 0 and model is not None:
                model_path = _save_model(ctl, msg, best_i, model)
        return {"dp_slices": out, "refit": best_i, "model_path": model_path}

    def _refit(self, a, ctl) -> Dict[str, Any]:
        msg = self.job_msg(a["seq"])
        dd = self.dataset(msg, ctl)
        t0 = time.perf_counter()
        model = refit_model(msg["plan"], msg["params"][a["candidate"]], dd)
        path = _save_model(ctl, msg, a["candidate"], model) if model is not None else None
        return {"model_path": path, "wall": time.perf_counter() - t0}


def _save_model(ctl, msg, cand: int, model) -> Optional[str]:
    try:
        model["job_id"] = msg["job_id"]
        model["subtask_id"] = msg["subtask_ids"][cand]
        if ctl is not None:
            model["feature_names"] = list(ctl.registry.load(msg["dataset_id"], msg["plan"]["feature_columns"],
                                                            msg["plan"]["target_column"]).feature_names)
            return ctl.models.save(f"{msg['subtask_ids'][cand]}_model", model)
        from ..engine.model_store import ModelStore

        return ModelStore(msg["models_root"]).save(f"{msg['subtask_ids'][cand]}_model", model)
    except Exception:
        traceback.print_exc()
        return None


def _private_client():
    """A second store connection for blocking waits (None: fall back to polling)."""
    try:
        return dist.service_client()
    except Exception:
        return None


class _null_ctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def collective_loop(core: WorkerCore, ctl: Optional[Controller] = None, start: int = 0) -> None:
    """An in-group rank's collective thread: runs the dispatcher's collective tasks
    (``coll/<i>``, from ``start``: dataset broadcasts, job score gathers) in order on the
    side group and its own stream while the worker thread keeps running slices.  A task
    every rank gave up together (``CollectiveAborted``: an OOM vote, a table rank 0 could
    not prepare) is answered and the thread goes on; any other failure means the
    communicator is unusable: the thread reports it and stops (the dispatcher re-forms the
    group, ``WorkerCore.regroup``)."""
    st = LockedStore(core.store._s, waiter=_private_client())
    stream = None
    if core.device.type == "cuda":
        torch.cuda.set_device(core.device)
        stream = torch.cuda.Stream(core.device)
    i = start
    while True:
        key = f"coll/{i}"
        try:
            while True:
                try:
                    st.wait([key], timeout=3600.0)
                    break
                except TimeoutError:
                    continue
            a = json.loads(st.get(key))
        except Exception:
            return
        if a["kind"] == "stop":
            return
        a["i"] = i
        failed = False
        try:
            out = core.collective(a, ctl, stream)
        except dist.CollectiveAborted as e:
            log.warning("worker %d: side task %d given up on every rank: %s", core.wid, i, e)
            out = {"error": f"{type(e).__name__}: {e}", "aborted": True}
        except Exception as e:
            traceback.print_exc()
            out, failed = {"error": f"{type(e).__name__}: {e}"}, True
        st.set(f"colldone/{core.wid}/{i}", json.dumps(json_safe(out)))
        st.add("coll/count", 1)
        post_wake(st)
        i += 1
        if failed:
            return


def post_wake(st: LockedStore) -> None:
    """Wake rank 0's dispatcher: ``wake/count`` numbers the events, ``wake/<n>`` is the key
    the dispatcher blocks on for the n-th one (TCPStore.wait, no timeout, no polling)."""
    n = int(st.add("wake/count", 1))
    st.set(f"wake/{n}", "1")


def post_result(st: LockedStore, wid: int, k: int, out: Dict[str, Any]) -> None:
    """Post a worker's answer: ``res/count`` numbers the answers (the dispatcher reads one
    counter instead of checking every busy worker's key), then wake the dispatcher."""
    st.set(f"res/{wid}/{k}", json.dumps(json_safe(out)))
    st.add("res/count", 1)
    post_wake(st)


def worker_loop(core: WorkerCore, ctl: Optional[Controller] = None, heartbeat: bool = True) -> None:
    """A worker's life: block until its next assignment, execute it, post the result.

    A device fault poisons this process's HIP context: the worker posts the error and
    exits non-zero; the dispatcher re-queues its slice to the survivors."""
    st, wid = core.store, core.wid
    hb = _Heartbeat(st, wid) if heartbeat else None
    core.start_collective_thread(ctl)   # this rank's collective thread (side group), when in a group
    k = 0
    try:
        while True:
            key = f"asg/{wid}/{k}"
            try:
                while True:
                    try:
                        st.wait([key], timeout=3600.0)
                        break
                    except TimeoutError:
                        continue
            except Exception:   # the store (hosted by rank 0) is gone: the service exited
                log.warning("worker %d lost the controller store; leaving", wid)
                return
            a = json.loads(st.get(key))
            st.delete_key(key)
            if a["kind"] == "stop":
                return
            try:
                out = core.execute(a, ctl)
            except Exception as e:
                traceback.print_exc()
                if is_device_fault(e):
                    post_result(st, wid, k, {"fatal": f"{type(e).__name__}: {e}"})
                    log.error("worker %d: device fault, exiting: %s", wid, e)
                    os._exit(3)
                out = {"error": f"{type(e).__name__}: {e}"}
            out["t_post"] = time.time()
            post_result(st, wid, k, out)
            k += 1
    finally:
        if hb is not None:
            hb.stop()


def staged_path(stage_dir: str, dataset_key: str) -> str:
    """Host staging file of a dataset (parallel/data.py stage_host: raw .npy + label sidecar)."""
    return os.path.join(stage_dir, f"{zlib.crc32(dataset_key.encode()) & 0xFFFFFFFF:08x}.npy")


def load_prep_timeout_s() -> float:
    """How long peers wait for rank 0 to parse / stage a table before a collective load
    (``DML_LOAD_PREP_TIMEOUT_S``, default 1800 s)."""
    return float(os.environ.get("DML_LOAD_PREP_TIMEOUT_S", "1800"))


def shard_load_min_bytes() -> int:
    """Tables of at least this many float32 bytes (``DML_SHARD_LOAD_MIN_MB``, default 1024) load
    sharded: rank 0 stages them once, each rank copies 1/N of the rows, one all-gather."""
    return int(float(os.environ.get("DML_SHARD_LOAD_MIN_MB", "1024")) * (1 << 20))


def needs_whole_rows(model_type: str, params: Dict[str, Any], gpu: bool = False) -> bool:
    """A candidate the row-sharded builders cannot fit exactly: absolute_error trees need
    per-node weighted medians over every row, and monotonic_cst's node bounds are not part of
    the row-sharded forest builder -- such a job runs task-parallel (never a silently
    different estimator; reference aws-prod/worker/worker.py:45,452 forwards params verbatim).
    GradientBoosting: the early-stopping validation split is not a sum over row shards; leaf
    percentiles (absolute_error / huber / quantile losses) are only on GPU workers (``gpu``),
    where the fused stage's radix select all-reduces its byte counts (models/boosting.py
    _sharded_stage) for trees of depth <= 10."""
    if model_type.startswith("GradientBoosting"):
        pct = params.get("loss") in ("absolute_error", "lad", "huber", "quantile")
        md = params.get("max_depth", 3)
        try:
            pct_ok = gpu and md is not None and int(md) <= 10
        except (TypeError, ValueError):   # a malformed depth fails that candidate in its own fit
            pct_ok = False
        return ((pct and not pct_ok)
                or bool(params.get("n_iter_no_change")) or params.get("monotonic_cst") is not None)
    if not model_type.startswith("RandomForest"):
        return False
    return params.get("criterion") == "absolute_error" or params.get("monotonic_cst") is not None


def _sharded_pct_ok() -> bool:
    from ..models.boosting import sharded_pct_ok

    return sharded_pct_ok()


def _binned_only_table(ctl: Controller, plan: Dict[str, Any], X, device) -> bool:
    """Same rule as the local device cache (engine/service.py DeviceCache._binned_only)."""
    if getattr(device, "type", str(device)) != "cuda" or not getattr(family_of(plan["model_type"]), "binned_ok", False):
        return False
    free = torch.cuda.mem_get_info(device)[0]
    return float(np.asarray(X).shape[0]) * np.asarray(X).shape[1] * 4 > ctl.config.stream_binned_fraction * free


def join_cluster(host: str, port: int, device: torch.device, mem_mb: int = 0, timeout_s: float = 60.0) -> int:
    """Join a running service as an extra worker (not a member of its process group): get
    a worker id from the dispatcher's store, announce it, and serve assignments until the
    service stops.  Datasets arrive host-staged; collectives are never asked of a joiner."""
    import datetime

    from torch.distributed import PrefixStore, TCPStore

    raw = TCPStore(host, port, is_master=False, timeout=datetime.timedelta(seconds=timeout_s))
    waiter = PrefixStore("dml", TCPStore(host, port, is_master=False, timeout=datetime.timedelta(seconds=timeout_s)))
    st = LockedStore(PrefixStore("dml", raw), waiter=waiter)   # the service's control plane (dist.service_store)
    n = int(st.add("join/n", 1))
    wid = MAX_WORKERS + n - 1
    st.set(f"join/{n - 1}", json.dumps({"wid": wid, "device": str(device), "mem_mb": mem_mb, "pid": os.getpid()}))
    core = WorkerCore(device, wid=wid, store=st, in_group=False)
    worker_loop(core, None)
    return wid


# ---------------------------------------------------------------------------------------
# rank 0: dispatcher
# ---------------------------------------------------------------------------------------
@dataclass
class _JobState:
    job: Job
    plan: Dict[str, Any]
    seq: int
    msg: Dict[str, Any]
    slices: List[List[int]]
    est: List[float]                        # estimated seconds per slice
    queue: Deque[int] = field(default_factory=collections.deque)
    inflight: Set[int] = field(default_factory=set)
    done: Dict[int, Any] = field(default_factory=dict)   # slice -> list[_Res]
    metrics: Dict[int, Dict[int, Any]] = field(default_factory=dict)
    mode: str = "task"                      # task | data
    transport: str = "rccl"                 # rccl (collective epoch) | staged (host file)
    staged_ready: bool = False
    held: Optional[int] = None              # the last slice, published after the refit
    refit_pending: bool = False
    refit_inflight: bool = False
    refit_candidate: int = -1
    finished: bool = False
    cand_costs: List[float] = field(default_factory=list)
    n_train: int = 0
    n_feat: int = 1
    rechunked: bool = False
    retired: Set[int] = field(default_factory=set)   # queued slices replaced by a re-cut
    scores_pending: bool = False            # waiting for the job's scores epoch (RCCL all-gather)
    scores_via: str = "store"               # where the final records' scores came from


@dataclass
class _Worker:
    wid: int
    in_group: bool
    next_k: int = 0
    busy: Optional[Dict[str, Any]] = None   # the in-flight assignment
    sent_at: float = 0.0
    est: float = 0.0
    loaded: Set[str] = field(default_factory=set)
    alive: bool = True
    joined_at: float = 0.0
    joined: bool = False                    # came in through join_cluster (not a launch rank)


class DistributedRunner(Runner):
    """Rank 0's dispatcher (runs in the main thread; the gateway serves from a thread and
    rank 0's own worker runs in another)."""

    def __init__(self, core: WorkerCore):
        self.core = core
        self.st = core.store
        self.pending: List[Job] = []
        self._cv = threading.Condition()
        self.seq = 0
        self.stop = False
        self.jobs: List[_JobState] = []
        inf = dist.info()
        self.world = inf.world
        self.workers: Dict[int, _Worker] = {r: _Worker(r, True) for r in range(self.world)}
        self.dead: Set[int] = set()
        self.session_used: Dict[str, float] = {}
        self.epoch: Optional[Dict[str, Any]] = None     # a collective epoch waiting for / holding the group
        self.epoch_queue: List[Dict[str, Any]] = []
        self._hb_missing_since: Dict[int, float] = {}
        self._joined = 0
        self._res_seen = 0                                 # answers consumed (res/count)
        self._wake_seen = 0                                # wake events consumed (wake/count)
        # collective tasks run by every in-group rank's collective thread (side group)
        self.coll_seq = 0
        self.coll_pending: Dict[int, Dict[str, Any]] = {}
        self._coll_seen = 0
        # side-group tasks held back while a collective epoch (default group) is queued or
        # running: the two communicators never have operations in flight at the same time, so
        # no rank can issue them in a different order than another (RCCL deadlock)
        self.coll_deferred: List[tuple] = []
        # a side collective failed or overran its deadline: no more collectives of any kind
        # (datasets host-staged, scores from the store copies, data-parallel jobs task-parallel)
        self.group_broken = False
        self._waiting = False                              # the dispatcher is blocked on a wake key
        self._next_liveness = self._next_membership = 0.0
        self._waiter = LockedStore(self.st._s, waiter=_private_client()) if isinstance(self.st, LockedStore) else None
        # control-plane accounting: dispatcher loop turns, answer -> next assignment latency
        self.stats: Dict[str, Any] = {"loops": 0, "answers": 0, "dispatch_latency_s": [], "max_drain_wait_s": 0.0}
        self._drain_since: Optional[float] = None        # an epoch is draining the group since
        self._t_answer: Dict[int, float] = {}
        self._stage_dir = os.environ.get("DML_STAGE_DIR") or (
            tempfile.mkdtemp(prefix="dml_stage_", dir="/dev/shm") if os.path.isdir("/dev/shm") else tempfile.mkdtemp())
        self._t0 = time.time()
        core.stage_dir = self._stage_dir   # rank 0's collective loads stage large tables here
        # communicator generations: after a rank death, a broken side collective or a new
        # member, rank 0 re-forms the process group over every live worker (regroup epoch)
        self.distributed = inf.is_dist
        self._backend = inf.backend
        self.gen = 0
        self._gen_next = 1
        self.regroup_enabled = os.environ.get("DML_REGROUP", "1") != "0"
        self.regroup_failures = 0
        self._regroup_after = 0.0
        self._regroup_drain_since: Optional[float] = None
        self._suspect: Set[int] = set()                    # never answered a regroup
        self._hb_age: Dict[int, float] = {}                # seconds since each worker's last heartbeat
        self.stats.update(regroups=0, regroup_failures=0, generation=0, stage_log=[])
        self.job_log: "collections.OrderedDict[str, Dict[str, Any]]" = collections.OrderedDict()
        # admission and host staging run OFF the dispatch thread (a 40 GB table's parse and
        # host write would stall every other job's dispatch): admission on one worker thread
        # (jobs keep their order), staging on two (a small table is not queued behind a
        # large one); results come back through queues the dispatcher drains
        from concurrent.futures import ThreadPoolExecutor

        self._admit_pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="dml-admit")
        self._stage_pool = ThreadPoolExecutor(max_workers=2, thread_name_prefix="dml-stage")
        self._admitted: "queue.Queue" = queue.Queue()
        self._staged_q: "queue.Queue" = queue.Queue()
        self._staging: Set[int] = set()
        self._admitting = 0

    def bind(self, controller: Controller) -> None:
        super().bind(controller)
        self.worker_ids = {r: controller.scheduler.register(f"rank{r}", 0, f"cuda:{r}") for r in range(self.world)}

    def submit(self, job: Job) -> None:
        with self._cv:
            self.pending.append(job)
            self._cv.notify_all()
        self._poke()

    def _poke(self) -> None:
        """Wake the dispatcher if it is blocked on the store (new job, shutdown, timer)."""
        if self._waiting:
            try:
                post_wake(self.st)
            except Exception:
                pass

    def _ticker(self) -> None:
        """Liveness / membership deadlines while the dispatcher blocks: one wake per 0.5 s."""
        while not self.stop:
            time.sleep(0.5)
            self._poke()

    def requeue(self, units) -> None:
        pass

    def shutdown(self) -> None:
        with self._cv:
            self.stop = True
            self._cv.notify_all()
        self._poke()

    # ---- main loop ---------------------------------------------------------------------
    def serve_forever(self, idle_poll_s: float = 0.05) -> None:
        # rank 0's process runs the dispatcher, the gateway, its own worker and the collective
        # thread: a 1 ms GIL switch interval (default 5 ms) bounds how long a worker thread's
        # Python stretch can hold an answer's dispatch back (config-5 rehearsal, 8 ranks:
        # profiles/r5_config5_8rank_gloo_dispatch.jsonl)
        import sys

        sys.setswitchinterval(float(os.environ.get("DML_GIL_SWITCH_S", "0.001")))
        w0 = threading.Thread(target=worker_loop, args=(self.core, self.ctl, False), daemon=True,
                              name="dml-rank0-worker")
        w0.start()
        threading.Thread(target=self._ticker, daemon=True, name="dml-dispatch-ticker").start()
        try:
            while True:
                with self._cv:
                    new = self.pending
                    self.pending = []
                    stopping = self.stop
                for job in new:
                    self._admit(job)
                self.stats["loops"] += 1
                busy = self._poll_admitted()
                busy = self._poll_staged() or busy
                busy = self._poll_results() or busy
                busy = self._poll_coll() or busy
                now = time.time()
                if now >= self._next_membership:
                    self._next_membership = now + 0.25
                    self._membership()
                if now >= self._next_liveness:
                    self._next_liveness = now + 0.5
                    self._liveness()
                self._dispatch()
                active = any(not js.finished for js in self.jobs) or self._admitting > 0 or any(
                    w.busy is not None and not w.busy.get("abandoned") for w in self.workers.values() if w.alive)
                if stopping and not active:
                    break
                if not active and not busy:
                    with self._cv:
                        if not self.pending and not self.stop:
                            self._cv.wait(timeout=idle_poll_s)
                elif not busy:
                    self._wait_answer(idle_poll_s)
        finally:
            if any(w.in_group for w in self.workers.values()) and self.core.side is not None:
                try:
                    self.st.set(f"coll/{self.coll_seq}", json.dumps({"kind": "stop"}))
                except Exception:
                    pass
            for w in self.workers.values():
                if w.alive:
                    self._assign(w, {"kind": "stop"})
            w0.join(timeout=30)
            self._admit_pool.shutdown(wait=False)
            self._stage_pool.shutdown(wait=True)
            self._cleanup_stage()

    # ---- admission -----------------------------------------------------------------------
    def _admit(self, job: Job) -> None:
        """Hand the job to the admission thread: the request is parsed and the table's
        metadata read (a first look at a large CSV counts its rows) there, not here."""
        self._admitting += 1
        self.stats.setdefault("submit_t", {})[job.job_id] = time.time()
        self._admit_pool.submit(self._prepare, job)

    def _prepare(self, job: Job) -> None:
        """(admission thread) everything about a job that does not touch dispatcher state."""
        try:
            plan = job_plan(job.request)
            meta = self.ctl.registry.metadata(job.dataset_id)
            key = dataset_key(self.ctl.registry, job.dataset_id, plan)
            self._admitted.put((job, (plan, meta, key), None))
        except Exception as e:
            self._admitted.put((job, None, e))
        self._poke()

    def _poll_admitted(self) -> bool:
        got = False
        while True:
            try:
                job, prep, err = self._admitted.get_nowait()
            except queue.Empty:
                return got
            got = True
            self._admitting -= 1
            if err is not None:
                traceback.print_exception(type(err), err, err.__traceback__)
                self._fail_job(job, err)
                continue
            self._admit_prepared(job, *prep)

    def _admit_prepared(self, job: Job, plan: Dict[str, Any], meta: Dict[str, Any], key: str) -> None:
        ctl = self.ctl
        try:
            n_rows = int(meta.get("n_rows", 1000))
            n_feat = max(1, int(meta.get("n_cols", 2)) - 1)
            todo = [sub.index for sub in job.subtasks if sub.status not in ("completed", "failed")]
            if not todo:
                return
            data_par = self._data_parallel(plan, len(todo), n_rows, n_feat)
            if data_par:
                gpu = getattr(self.core.device, "type", "") == "cuda" and _sharded_pct_ok()
                whole = [i for i in todo if needs_whole_rows(plan["model_type"], job.subtasks[i].spec["parameters"],
                                                             gpu=gpu)]
                if whole:   # never a silently different model: such a job runs task-parallel
                    log.warning("job %s: %d candidate(s) need every row on one rank (absolute_error / "
                                "monotonic_cst): task-parallel instead of row-sharded", job.job_id, len(whole))
                    data_par = False
            slices = plan_slices(ctl, plan, todo, int(n_rows * 0.8), n_feat, 2,
                                 min_slices=1 if data_par else min(len(todo), 2 * self._n_alive()))
            costs = candidate_costs(plan, int(n_rows * 0.8), n_feat, 2)
            est = [ctl.scheduler.estimate(plan["model_type"], sum(costs[i] for i in ids)) for ids in slices]
            seq = self.seq
            self.seq += 1
            msg = {"job_id": job.job_id, "session_id": job.session_id, "dataset_id": job.dataset_id,
                   "dataset_key": key, "plan": plan,
                   "slices": slices, "params": [sub.spec["parameters"] for sub in job.subtasks],
                   "subtask_ids": [sub.subtask_id for sub in job.subtasks], "seed": job_seed(job.job_id),
                   "keep_models": ctl.config.keep_models, "models_root": ctl.models.root}
            js = _JobState(job, plan, seq, msg, slices, est, mode="data" if data_par else "task",
                           cand_costs=costs, n_train=int(n_rows * 0.8), n_feat=n_feat)
            js.queue.extend(range(len(slices)))
            # datasets travel by collective broadcast while the whole group is alive and
            # nobody joined from outside it; otherwise host-staged
            # (DML_TRANSPORT=staged: always host-staged, e.g. a host whose xGMI is shared)
            js.transport = "rccl" if (self._group_ok() and os.environ.get("DML_TRANSPORT") != "staged") else "staged"
            if js.transport == "staged" or self._joiners_alive():
                self._stage(js)
            self._publish_msg(js)
            for ids in slices:
                ctl.table.mark_running(job.job_id, ids, "cluster")
            self.jobs.append(js)
            self.session_used.setdefault(job.session_id, 0.0)
            if js.mode == "data":
                self.epoch_queue.append({"kind": "dp", "job": js})
            self._log_job(js)
        except Exception as e:
            traceback.print_exc()
            self._fail_job(job, e)

    def _publish_msg(self, js: _JobState) -> None:
        self.st.set(f"job/{js.seq}", json.dumps(json_safe(js.msg)))

    def _stage(self, js: _JobState) -> None:
        """Ask the staging thread for the job's host-staged table (non-blocking): its slices
        are handed out once ``_poll_staged`` sees the file (``staged_ready``)."""
        if js.staged_ready or js.seq in self._staging:
            return
        self._staging.add(js.seq)
        path = staged_path(self._stage_dir, js.msg["dataset_key"])
        reg, ds_id, fc, tc = self.ctl.registry, js.job.dataset_id, js.plan["feature_columns"], js.plan["target_column"]

        def load():
            ds = reg.load(ds_id, fc, tc)
            return ds.X, ds.y

        def work():
            t0 = time.time()
            try:
                faults.maybe_delay_staging()
                pdata.ensure_staged(load, path, pin=True)
                self._staged_q.put((js, path, None))
            except Exception as e:
                self._staged_q.put((js, path, e))
            nbytes = os.path.getsize(path) if os.path.exists(path) else 0
            self.stats["stage_log"].append((js.job.job_id, t0, time.time(), nbytes))
            self._poke()

        self._stage_pool.submit(work)

    def _poll_staged(self) -> bool:
        got = False
        while True:
            try:
                js, path, err = self._staged_q.get_nowait()
            except queue.Empty:
                return got
            got = True
            self._staging.discard(js.seq)
            if js.finished:
                continue
            if err is not None:
                log.error("host staging of %s failed: %s", js.job.dataset_id, err)
                self._fail_job(js.job, err)
                js.finished = True
                self._cleanup_job(js)
                continue
            js.msg["staged"] = path
            js.staged_ready = True
            self._publish_msg(js)
            ent = self.job_log.get(js.job.job_id)
            if ent is not None:
                ent["staged_t"] = time.time()

    def _group_ok(self) -> bool:
        """Collectives may be issued: a process group exists and nothing broke it since the
        current generation formed."""
        return self.distributed and dist.info().is_dist and not self.dead and not self.group_broken

    def _log_job(self, js: _JobState) -> None:
        """Per-job transport / mode / generation (cluster_info; bounded)."""
        ent = self.job_log.setdefault(js.job.job_id, {"admitted_t": time.time()})
        ent.update(transport=js.transport, mode=js.mode, generation=self.gen, scores_via=js.scores_via)
        while len(self.job_log) > 256:
            self.job_log.popitem(last=False)

    def cluster_info(self) -> Dict[str, Any]:
        """The collective plane's state (/health): generation, members, regroup counters and
        the last jobs' transport."""
        return {"generation": self.gen, "world": self.world, "group_ok": self._group_ok(),
                "members": sorted(w.wid for w in self.workers.values() if w.alive and w.in_group),
                "workers": sorted(w.wid for w in self.workers.values() if w.alive),
                "regroups": self.stats["regroups"], "regroup_failures": self.stats["regroup_failures"],
                "jobs": dict(self.job_log)}

    def _cleanup_stage(self) -> None:
        import shutil

        if not os.environ.get("DML_STAGE_DIR"):
            shutil.rmtree(self._stage_dir, ignore_errors=True)

    def _data_parallel(self, plan, n_todo: int, n_rows: int, n_feat: int) -> bool:
        """Row-sharded data parallelism needs every rank of the group: never once one died."""
        par = plan.get("parallelism", "auto")
        if par == "task" or not self._group_ok() or \
                not getattr(family_of(plan["model_type"]), "data_parallel", False):
            return False
        if par == "data":
            return True
        cfg = self.ctl.config
        cells = n_rows * n_feat
        # forests: only for tables too large to replicate (a per-level all-reduce costs more
        # than it saves while every rank can hold the table and run whole fits)
        few = n_todo < self.world and getattr(family_of(plan["model_type"]), "dp_when_few", True)
        return cells >= cfg.dp_min_cells and (few or cells * 4 > cfg.dp_auto_gb * 2 ** 30)

    def _fail_job(self, job: Job, e: Exception) -> None:
        for sub in job.subtasks:
            if sub.status not in ("completed", "failed"):
                self.ctl.table.finish_subtask(job.job_id, sub.subtask_id, "failed", error=f"{type(e).__name__}: {e}")

    # ---- assignments -----------------------------------------------------------------------
    def _n_alive(self) -> int:
        return sum(1 for w in self.workers.values() if w.alive)

    def _joiners_alive(self) -> bool:
        return any(w.alive and not w.in_group for w in self.workers.values())

    def _assign(self, w: _Worker, a: Dict[str, Any], est: float = 0.0) -> None:
        k = w.next_k
        w.next_k += 1
        t_ans = self._t_answer.pop(w.wid, None)
        if t_ans is not None and a["kind"] == "slice":   # the worker's answer -> its next slice
            lat = self.stats["dispatch_latency_s"]
            lat.append(time.time() - t_ans)
            if len(lat) > 100000:
                del lat[:50000]
        if a["kind"] != "stop":
            w.busy = dict(a, k=k)
            w.sent_at = time.time()
            w.est = est
        self.st.set(f"asg/{w.wid}/{k}", json.dumps(a))

    def _dispatch(self) -> None:
        # a collective epoch owns the process group until every rank has answered
        if self.epoch is not None:
            return
        if self._regroup_due() and self._regroup_step():
            return   # re-forming the group (draining its members first)
        if not self.epoch_queue and self.coll_deferred:
            self._flush_coll()
        if self.epoch_queue:
            ep = self.epoch_queue[0]
            js = ep["job"]
            group = [w for w in self.workers.values() if w.in_group]
            if not self._group_ok() or any(not w.alive for w in group):
                # the group is broken (and will not be re-formed): a data-parallel job runs
                # task-parallel instead
                self.epoch_queue.pop(0)
                if ep["kind"] == "dp":
                    js.mode = "task"
                    if js.transport == "rccl":
                        js.transport = "staged"
                        self._stage(js)
                elif ep["kind"] == "scores":   # no collective any more: the store copies stand
                    js.scores_pending = False
                    self._complete(js)
                return
            # the epoch's collectives (default group) start only once no side-group task is in
            # flight; new side tasks are deferred meanwhile (_post_coll)
            if all(w.busy is None for w in group) and not self.coll_pending:
                if self._drain_since is not None:
                    self.stats["max_drain_wait_s"] = max(self.stats["max_drain_wait_s"],
                                                         time.time() - self._drain_since)
                    self._drain_since = None
                self.epoch_queue.pop(0)
                self.epoch = {"kind": ep["kind"], "job": js, "waiting": {w.wid for w in group}}
                payload = {"kind": ep["kind"], "seq": js.seq}
                if ep["kind"] == "scores":
                    payload.update(n=len(js.job.subtasks), width=score_width(js.plan))
                for w in group:
                    self._assign(w, payload)
                return
            if self._drain_since is None and any(w.busy is None for w in group):
                self._drain_since = time.time()   # idle ranks wait for the epoch from here
            return   # drain: no new slices until the group is idle
        # refits go to rank 0 (it owns the controller and saves the artefact)
        w0 = self.workers[0]
        for js in self.jobs:
            if js.refit_pending and w0.busy is None:
                key = js.msg["dataset_key"]
                if key not in w0.loaded and js.transport == "rccl":
                    self._request_load(js)
                    return
                if key not in w0.loaded and js.transport != "rccl" and not js.staged_ready:
                    self._stage(js)
                    continue
                self._assign(w0, {"kind": "refit", "seq": js.seq, "candidate": js.refit_candidate})
                js.refit_pending = False
                js.refit_inflight = True
        for w in sorted(self.workers.values(), key=lambda w: w.wid):
            if not w.alive or w.busy is not None:
                continue
            js, i = self._next_slice(w)
            if js is None:
                # nothing this worker can run yet: the dispatch-latency clock (answer -> next
                # slice) restarts, so idle time without runnable work is not counted as latency
                if w.wid in self._t_answer:
                    self._t_answer[w.wid] = time.time()
                if self.epoch_queue:
                    return
                continue
            js.queue.remove(i)
            js.inflight.add(i)
            est = js.est[i]
            self.session_used[js.job.session_id] = self.session_used.get(js.job.session_id, 0.0) + est
            self._assign(w, {"kind": "slice", "seq": js.seq, "slice": i, "ids": js.slices[i]}, est)
            ent = self.job_log.get(js.job.job_id)
            if ent is not None and "first_slice_t" not in ent:
                ent["first_slice_t"] = time.time()

    def _next_slice(self, w: _Worker):
        """Fair share: the next slice comes from the job of the least-served session (ties:
        admission order) among the jobs this worker can run now."""
        cands = []
        for js in self.jobs:
            if js.finished or js.mode != "task" or not js.queue:
                continue
            key = js.msg["dataset_key"]
            if key not in w.loaded:
                if js.transport == "rccl" and w.in_group:
                    self._request_load(js)
                    continue
                if not js.staged_ready:   # the staging thread publishes it; other jobs meanwhile
                    self._stage(js)
                    continue
            cands.append(js)
        if not cands:
            return None, None
        js = min(cands, key=lambda j: (self.session_used.get(j.job.session_id, 0.0), j.seq))
        return js, js.queue[0]

    def _request_load(self, js: _JobState) -> None:
        """Broadcast the job's table to every in-group rank -- a collective task of the
        ranks' collective threads, so no rank is drained for it."""
        key = js.msg["dataset_key"]
        if any(t["kind"] == "load" and t["dkey"] == key for t in self.coll_pending.values()):
            return
        self._post_coll({"kind": "load", "seq": js.seq}, js, dkey=key)

    def _post_coll(self, task: Dict[str, Any], js: _JobState, dkey: str = "") -> None:
        if self.group_broken:
            self._coll_fallback(task["kind"], js)
            return
        if self.epoch is not None or self.epoch_queue:
            if not any(t[0]["kind"] == task["kind"] and t[1] is js for t in self.coll_deferred):
                self.coll_deferred.append((task, js, dkey))
            return
        i = self.coll_seq
        self.coll_seq += 1
        self.st.set(f"coll/{i}", json.dumps(task))
        self.coll_pending[i] = {"kind": task["kind"], "job": js, "dkey": dkey, "t0": time.time(),
                                "waiting": {w.wid for w in self.workers.values() if w.in_group and w.alive}}

    def _flush_coll(self) -> None:
        """Post the side-group tasks deferred while a collective epoch held the group."""
        todo, self.coll_deferred = self.coll_deferred, []
        for task, js, dkey in todo:
            if not js.finished:
                self._post_coll(task, js, dkey)

    def _coll_fallback(self, kind: str, js: _JobState) -> None:
        """A side-group task that can no longer run: a load becomes host staging, a scores
        gather leaves the per-slice store copies standing."""
        if kind == "load":
            if js.transport == "rccl":
                js.transport = "staged"
            self._stage(js)
        elif kind == "scores" and js.scores_pending:
            js.scores_pending = False
            js.scores_via = "store-fallback"
            self._complete(js)

    def _break_group(self, why: str) -> None:
        """The side communicator failed (a collective raised or overran its deadline: a rank
        is dead, hung, or out of memory): no rank issues another collective.  Every pending
        and deferred side task falls back, every job that counted on RCCL is host-staged.
        Safe to call more than once."""
        first = not self.group_broken
        self.group_broken = True
        self._membership_changed()
        if first:
            log.error("process group broken (%s): host staging and store copies until it is re-formed", why)
        pending = [(t["kind"], t["job"]) for t in self.coll_pending.values()]
        pending += [(task["kind"], js) for task, js, _ in self.coll_deferred]
        # the abandoned tasks' store keys: a posted task becomes a stop (a collective thread
        # that has not reached it yet exits instead of entering a collective on the broken
        # group) and answers already written are dropped (a later one is never read)
        for i, t in self.coll_pending.items():
            try:
                self.st.set(f"coll/{i}", json.dumps({"kind": "stop"}))
                for wid in t.get("waiting", ()):
                    self.st.delete_key(f"colldone/{wid}/{i}")
            except Exception:  # pragma: no cover - store gone with the service
                pass
        self.coll_pending.clear()
        self.coll_deferred = []
        for kind, js in pending:
            self._coll_fallback(kind, js)
        for js in self.jobs:
            if not js.finished and js.transport == "rccl":
                js.transport = "staged"
                self._stage(js)

    def _poll_coll(self) -> bool:
        """Answers of the collective threads (``colldone/<worker>/<task>``)."""
        n = int(self.st.add("coll/count", 0))
        if n == self._coll_seen:
            return False
        self._coll_seen = n
        for i, t in list(self.coll_pending.items()):
            for wid in list(t["waiting"]):
                key = f"colldone/{wid}/{i}"
                if not self.st.check([key]):
                    continue
                out = json.loads(self.st.get(key))
                self.st.delete_key(key)
                t["waiting"].discard(wid)
                self._on_coll(t, wid, out)
            if not t["waiting"]:
                self.coll_pending.pop(i, None)
                self.st.delete_key(f"coll/{i}")
        return True

    def _on_coll(self, t: Dict[str, Any], wid: int, out: Dict[str, Any]) -> None:
        js, w = t["job"], self.workers.get(wid)
        if "error" in out and out.get("aborted"):
            # every rank gave this task up together before the collective (OOM vote, table
            # preparation failed): the communicator is intact; this job's table is
            # host-staged instead and the worker that could not take it re-plans its slices
            # on its own (host copy, bounded retries)
            if t["kind"] == "load" and js.transport == "rccl":
                log.warning("collective load of %s given up on every rank (%s): host-staging this job only",
                            js.job.dataset_id, out["error"])
                js.transport = "staged"
                self._stage(js)
                self._log_job(js)
            elif t["kind"] == "scores" and wid == 0:
                self._coll_fallback("scores", js)
            return
        if "error" in out:
            # the failing rank's collective thread has stopped and its peers are (or will be)
            # stuck in this collective until the side timeout: the group is broken until the
            # dispatcher re-forms it (_regroup_step)
            self._break_group(f"{t['kind']} collective failed on worker {wid}: {out['error']}")
            return
        if t["kind"] == "load":
            if w is not None and "cache" in out:
                w.loaded = set(out["cache"])
            if "error" in out and js.transport == "rccl":
                log.error("collective load of %s failed on worker %d (%s): host-staging it", js.job.dataset_id, wid,
                          out["error"])
                js.transport = "staged"
                self._stage(js)
            return
        if t["kind"] == "scores" and wid == 0 and js.scores_pending:
            if "error" in out:
                log.error("scores gather of job %s failed (%s): the store copies stand", js.job.job_id, out["error"])
            else:
                self._merge_scores(js)
            js.scores_pending = False
            self._complete(js)

    # ---- results ----------------------------------------------------------------------------
    def _wait_answer(self, timeout: float) -> None:
        """Block (server-side, on a private store client) until the next wake event: a
        worker answer, a submitted job, shutdown, or the 0.5 s liveness ticker -- no busy
        polling of every worker's result key."""
        if self._waiter is None or self._waiter._waiter is None:
            time.sleep(POLL_S)
            return
        self._waiting = True
        try:
            with self._cv:
                if self.pending or self.stop:
                    return
            self._waiter.wait([f"wake/{self._wake_seen + 1}"], timeout=30.0)
        except TimeoutError:
            pass
        except Exception:
            time.sleep(POLL_S)
        finally:
            self._waiting = False
            m = int(self.st.add("wake/count", 0))
            for i in range(self._wake_seen + 1, m + 1):
                self.st.delete_key(f"wake/{i}")
            self._wake_seen = m

    def store_ops(self) -> int:
        """Store operations issued by rank 0's clients (dispatcher, its worker, heartbeat)."""
        return int(getattr(self.st, "ops", 0)) + int(getattr(self._waiter, "ops", 0))

    def _poll_results(self) -> bool:
        n = int(self.st.add("res/count", 0))
        if n == self._res_seen:
            return False
        self._res_seen = n
        got = False
        for w in list(self.workers.values()):
            if w.busy is None:
                continue
            key = f"res/{w.wid}/{w.busy['k']}"
            if not self.st.check([key]):
                continue
            out = json.loads(self.st.get(key))
            self.st.delete_key(key)
            a = w.busy
            w.busy = None
            got = True
            self.stats["answers"] += 1
            self._t_answer[w.wid] = float(out.get("t_post", time.time()))
            # control-plane lag: a worker's answer posted -> consumed by the dispatcher (the
            # dispatch latency above also counts time the worker waited for queued work)
            lag = self.stats.setdefault("answer_lag_s", [])
            lag.append(max(0.0, time.time() - self._t_answer[w.wid]))
            if len(lag) > 100000:
                del lag[:50000]
            if "fatal" in out:
                log.error("worker %d reported a device fault (%s): re-queueing its work", w.wid, out["fatal"])
                self._declare_dead(w, a)
                continue
            self._on_result(w, a, out)
        return got

    def _on_result(self, w: _Worker, a: Dict[str, Any], out: Dict[str, Any]) -> None:
        kind = a["kind"]
        if kind == "regroup":
            self._suspect.discard(w.wid)
            ep = self.epoch
            if ep is not None and ep["kind"] == "regroup" and ep["gen"] == a["gen"]:
                if "error" in out:
                    ep["failed"][w.wid] = out["error"]
                else:
                    ep["ok"].add(w.wid)
                self._epoch_answer(w)
            return
        js = self._job(a.get("seq"))
        if kind == "load":
            if "cache" in out:
                w.loaded = set(out["cache"])
            if "error" in out and js is not None and js.transport == "rccl":
                log.error("collective load of %s failed on worker %d (%s): host-staging it", js.job.dataset_id,
                          w.wid, out["error"])
                js.transport = "staged"
                self._stage(js)
            self._epoch_answer(w)
            return
        if kind == "dp":
            if w.wid == 0 and js is not None and "error" in out:
                self._dp_failed(js, out["error"])
                return
            self._epoch_answer(w)
            if w.wid == 0 and js is not None:
                self._finish_dp(js, out)
            return
        if kind == "scores":
            self._epoch_answer(w)
            if w.wid == 0 and js is not None:
                if "error" in out:
                    log.error("scores epoch of job %s failed (%s): the store copies stand", js.job.job_id, out["error"])
                else:
                    self._merge_scores(js)
                js.scores_pending = False
                self._complete(js)
            return
        if js is None:
            return
        if kind == "refit":
            js.refit_inflight = False
            self._finish_job(js, out.get("model_path"))
            return
        # slice
        i = a["slice"]
        js.inflight.discard(i)
        if "cache" in out:
            w.loaded = set(out["cache"])
        if "error" in out:   # the whole slice raised outside the executor: its candidates fail
            res = [_Res({"candidate": c, "ok": False, "error": out["error"]}) for c in a["ids"]]
            metrics = {}
        else:
            res = [_Res(d) for d in out["results"]]
            metrics = {d["candidate"]: d.get("metrics") for d in out["results"]}
        wall = float(out.get("wall", 0.0))
        sid = js.job.session_id
        self.session_used[sid] = self.session_used.get(sid, 0.0) - w.est + wall
        try:
            from ..engine.scheduler import Unit

            cost = sum(js.cand_costs[c] for c in a["ids"]) if js.cand_costs else 1.0
            self.ctl.scheduler.observe(self.worker_ids.get(w.wid, f"rank{w.wid}"),
                                       Unit(unit_id=f"{js.job.job_id}:{i}", cost=cost, algo=js.job.model_type), wall)
        except Exception:
            pass
        if "error" not in out and (not js.rechunked or should_recut(
                self.ctl, js.plan, [js.slices[q] for q in js.queue], js.cand_costs)):
            self._rechunk(js)
        if i in js.done:   # a re-queued slice finished twice: count it once
            return
        js.done[i] = res
        js.metrics[i] = metrics
        if len(js.done) + len(js.retired) < len(js.slices):
            publish_results(self.ctl, js.job, res, metrics)
            return
        js.held = i
        self._complete(js)

    def _rechunk(self, js: _JobState) -> None:
        """The job was cut with the prior seconds-per-cost; its first slices calibrated the
        cost model: re-cut the still-queued candidates into ~chunk_target_s slices (a
        one-candidate GPU batch leaves most of the chip idle at the top levels).  Runs
        after the first slice and again whenever the queue, priced with the current
        calibration, drifts far from the target (``should_recut``)."""
        js.rechunked = True
        queued = list(js.queue)
        if len(queued) < 2:
            return
        ids = [c for q in queued for c in js.slices[q]]
        new = plan_slices(self.ctl, js.plan, ids, js.n_train, js.n_feat, 2, min_slices=min(len(ids), self._n_alive()))
        base = len(js.slices)
        js.slices.extend(new)
        js.est.extend(self.ctl.scheduler.estimate(js.plan["model_type"], sum(js.cand_costs[c] for c in sl))
                      for sl in new)
        js.retired.update(queued)
        js.queue = collections.deque(range(base, base + len(new)))

    def _collective_scores(self, js: _JobState) -> bool:
        """The job's scores can travel by collective: the whole launch group is alive and
        every slice ran inside it."""
        return (js.transport == "rccl" and self._group_ok()
                and js.scores_via == "store"
                and all(w.alive for w in self.workers.values() if w.in_group))

    def _merge_scores(self, js: _JobState) -> None:
        """The final records' scores from the all-gathered table: the held slice's results
        before they are published, the already-published subtasks in the job table."""
        got = self.core.gathered.pop(js.seq, None)
        if got is None:
            return
        tab, backend = got
        via = "rccl" if backend == "nccl" else str(backend)   # nccl IS RCCL on ROCm
        W = tab.shape[1] - 1
        mismatch = 0
        for i, res in js.done.items():
            for r in res:
                row = tab[r.candidate] if 0 <= r.candidate < tab.shape[0] else None
                if row is None or row[W] == 0 or not r.ok or row[0] != 1.0:
                    continue
                ncv = int(row[3])
                upd = {"mean_cv_score": float(row[1]), "std_cv_score": float(row[2]),
                       "cv_scores": [float(v) for v in row[SCORE_HEAD:SCORE_HEAD + ncv]], "scores_via": via}
                old = r.result or {}
                if any(json.dumps(json_safe(old.get(k))) != json.dumps(json_safe(v))
                       for k, v in upd.items() if k != "scores_via"):
                    mismatch += 1
                r.result = dict(old, **upd)
                if i != js.held:
                    self.ctl.table.update_result(js.job.job_id, js.job.subtasks[r.candidate].subtask_id, upd)
        js.scores_via = via
        if mismatch:
            log.error("job %s: %d candidates' collective scores differ from their store copies", js.job.job_id,
                      mismatch)

    def _complete(self, js: _JobState) -> None:
        """Every slice is in: all-gather the scores (scores epoch), refit the winner (on
        rank 0), then publish the held slice."""
        if self._collective_scores(js):
            if not js.scores_pending:
                js.scores_pending = True
                self._post_coll({"kind": "scores", "seq": js.seq, "n": len(js.job.subtasks),
                                 "width": score_width(js.plan)}, js)
            return
        best = pick_refit(self.ctl, js.job, js.plan, js.done[js.held])
        if best is None:
            self._finish_job(js, None)
            return
        js.refit_candidate = best
        js.refit_pending = True

    def _finish_job(self, js: _JobState, model_path: Optional[str]) -> None:
        if model_path and js.refit_candidate >= 0:
            attach_model(self.ctl, js.job, js.done.get(js.held, []), js.refit_candidate, model_path)
        if js.held is not None:
            publish_results(self.ctl, js.job, js.done[js.held], js.metrics.get(js.held, {}))
        js.finished = True
        self._cleanup_job(js)

    def _dp_failed(self, js: _JobState, err: str) -> None:
        """A data-parallel epoch failed (a collective timed out on a dead or hung member, or
        raised): the reference re-places a lost worker's tasks and keeps serving
        (aws-prod/scheduler/scheduler_service.py:205-247).  Here the epoch is abandoned at
        once -- ranks still inside it answer when their own collective times out; a hung one
        never does and simply gets no more work -- the group is broken for good (no rank
        issues another collective), and the job is re-cut and re-run TASK-parallel on the
        survivors from the host-staged table.  Nothing of the failed epoch was published."""
        log.error("data-parallel epoch of job %s failed (%s): re-running it task-parallel on the survivors",
                  js.job.job_id, err)
        if self.epoch is not None:
            for wid in self.epoch["waiting"]:
                ww = self.workers.get(wid)
                if ww is not None and ww.busy is not None:
                    ww.busy["abandoned"] = True   # its late answer frees it; a hung rank stays parked
            self.epoch = None
        self._break_group(f"data-parallel epoch failed: {err}")
        ids = [c for sl in js.slices for c in sl]
        js.slices = plan_slices(self.ctl, js.plan, ids, js.n_train, js.n_feat, 2,
                                min_slices=min(len(ids), 2 * max(1, self._n_alive())))
        js.est = [self.ctl.scheduler.estimate(js.plan["model_type"], sum(js.cand_costs[c] for c in sl))
                  for sl in js.slices]
        js.queue = collections.deque(range(len(js.slices)))
        js.inflight.clear()
        js.done.clear()
        js.metrics.clear()
        js.retired.clear()
        js.rechunked = True
        js.mode = "task"
        js.transport = "staged"
        js.msg["slices"] = js.slices
        self._publish_msg(js)
        self._stage(js)
        self._log_job(js)
        self.stats["dp_requeued"] = self.stats.get("dp_requeued", 0) + 1

    def _finish_dp(self, js: _JobState, out: Dict[str, Any]) -> None:
        if "error" in out:   # (rank 0's error answers go through _dp_failed)
            self._dp_failed(js, out["error"])
            return
        slices = out.get("dp_slices", [])
        best_i, path = out.get("refit", -1), out.get("model_path")
        for n, sl in enumerate(slices):
            res = [_Res(d) for d in sl["results"]]
            metrics = {d["candidate"]: d.get("metrics") for d in sl["results"]}
            if path:
                for x in res:
                    if x.candidate == best_i and x.ok:
                        x.result["model_path"] = path
            js.done[n] = res
            publish_results(self.ctl, js.job, res, metrics)
        js.finished = True
        self._cleanup_job(js)

    def _epoch_answer(self, w: _Worker) -> None:
        if self.epoch is None:
            return
        self.epoch["waiting"].discard(w.wid)
        if not self.epoch["waiting"]:
            ep, self.epoch = self.epoch, None
            if ep["kind"] == "regroup":
                self._finish_regroup(ep)
            if not self.epoch_queue and self.coll_deferred:
                self._flush_coll()

    def _job(self, seq) -> Optional[_JobState]:
        if seq is None:
            return None
        for js in self.jobs:
            if js.seq == seq:
                return js
        return None

    def _cleanup_job(self, js: _JobState) -> None:
        if js.job.job_id in self.job_log:
            self.job_log[js.job.job_id]["scores_via"] = js.scores_via
        self.st.delete_key(f"job/{js.seq}")
        self.st.delete_key(f"job/{js.seq}/refit")
        self.jobs = [j for j in self.jobs if not j.finished]

    # ---- membership and liveness ------------------------------------------------------------
    def _membership(self) -> None:
        """Workers that joined from outside the process group (join_cluster)."""
        try:
            n = int(self.st.add("join/n", 0))
        except Exception:
            return
        while self._joined < n:
            key = f"join/{self._joined}"
            if not self.st.check([key]):
                return
            info = json.loads(self.st.get(key))
            wid = int(info["wid"])
            self.workers[wid] = _Worker(wid, False, joined_at=time.time(), joined=True)
            self.worker_ids[wid] = self.ctl.scheduler.register(f"rank{wid}", int(info.get("mem_mb", 0)),
                                                               info.get("device", "cpu"))
            log.info("worker %d joined (%s)", wid, info.get("device"))
            self._joined += 1
            self._membership_changed()   # the next generation takes the joiner in
            for js in self.jobs:   # until then it reads host-staged datasets
                if not js.finished and not js.staged_ready:
                    self._stage(js)

    def join_info(self) -> Optional[Dict[str, Any]]:
        """The rendezvous store a ``join_cluster`` worker connects to (/subscribe answer)."""
        return {"host": os.environ.get("MASTER_ADDR", "127.0.0.1"), "port": int(os.environ.get("MASTER_PORT", "0")),
                "workers": sum(1 for w in self.workers.values() if w.alive)}

    def leave(self, worker_id: str) -> bool:
        for wid, sid in list(self.worker_ids.items()):
            if sid == worker_id:
                return self.remove_worker(wid)
        return False

    def remove_worker(self, wid: int) -> bool:
        """Graceful leave (/unsubscribe): finish the current assignment, get no more."""
        w = self.workers.get(wid)
        if w is None or not w.alive or not w.joined:
            return False
        self._assign(w, {"kind": "stop"})
        w.alive = False
        if w.in_group:   # it was a member of the current generation: re-form without it
            w.in_group = False
            self._break_group(f"worker {wid} left")
        return True

    def _liveness(self) -> None:
        now = time.time()
        for w in list(self.workers.values()):
            if w.wid == 0 or not w.alive:
                continue
            try:
                hb = float(self.st.get(f"hb/{w.wid}")) if self.st.check([f"hb/{w.wid}"]) else None
            except Exception:
                hb = now
            if hb is None:   # never beat: silent since we first looked
                hb = self._hb_missing_since.setdefault(w.wid, now)
            self._hb_age[w.wid] = now - hb
            if now - hb > self.ctl.config.dead_after_s:
                log.warning("worker %d missed heartbeats for %.1fs: declared dead", w.wid, now - hb)
                self._declare_dead(w, w.busy)
            else:
                self.ctl.scheduler.heartbeat(self.worker_ids.get(w.wid, ""))
        self.ctl.scheduler.heartbeat(self.worker_ids.get(0, ""))
        # a side task no rank answered within its deadline (its peers' blocking waits time out
        # after side_timeout_s; a collective thread that died silently never answers)
        limit = dist.side_timeout_s() + float(os.environ.get("DML_COLL_GRACE_S", "30"))
        late = [i for i, t in self.coll_pending.items() if now - t["t0"] > limit]
        if late:
            self._break_group(f"side collective task(s) {late} unanswered after {limit:.0f}s")
        ep = self.epoch
        if ep is not None and ep["kind"] == "regroup" and \
                now - ep["t0"] > dist.regroup_timeout_s() + float(os.environ.get("DML_COLL_GRACE_S", "30")):
            for wid in list(ep["waiting"]):   # never answered: hung; excluded from the next try
                ww = self.workers.get(wid)
                if ww is not None and ww.busy is not None:
                    ww.busy["abandoned"] = True
                ep["failed"][wid] = "no answer"
                self._suspect.add(wid)
            ep["waiting"].clear()
            self.epoch = None
            self._finish_regroup(ep)

    def _declare_dead(self, w: _Worker, a: Optional[Dict[str, Any]]) -> None:
        w.alive = False
        w.busy = None
        self._membership_changed()
        if self.epoch is not None and self.epoch["kind"] == "regroup" and w.wid in self.epoch["waiting"]:
            self.epoch["failed"][w.wid] = "died"
        if w.in_group:
            self.dead.add(w.wid)
        self.ctl.scheduler.unsubscribe(self.worker_ids.get(w.wid, ""))
        if a is not None and a["kind"] == "slice":
            js = self._job(a["seq"])
            if js is not None and a["slice"] not in js.done:
                js.inflight.discard(a["slice"])
                js.queue.appendleft(a["slice"])   # re-queued first: it has waited longest
        if self.epoch is not None:
            # a collective cannot complete without this rank: the survivors of the epoch time
            # out (DML_COLLECTIVE_TIMEOUT_S); the dispatcher stops waiting for the dead one
            self._epoch_answer(w)
        if w.in_group:
            # pending side-group collectives can no longer complete: loads fall back to
            # host staging, score gathers to the per-slice store copies; the group is broken
            # for good (pending collectives become host-staged / task-parallel)
            self._break_group(f"worker {w.wid} died")

    # ---- communicator generations ------------------------------------------------------------
    def _membership_changed(self) -> None:
        """A member died, left, joined or broke a collective: re-form the group soon (a short
        delay batches a death with the respawn that follows it)."""
        self._regroup_after = max(self._regroup_after, time.time() + float(os.environ.get("DML_REGROUP_DELAY_S", "1")))

    def _regroup_due(self) -> bool:
        if not (self.distributed and self.regroup_enabled):
            return False
        if self.regroup_failures >= int(os.environ.get("DML_REGROUP_MAX_FAILURES", "5")):
            return False
        if time.time() < self._regroup_after:
            return False
        return self.group_broken or bool(self.dead) or any(
            not w.in_group for w in self.workers.values() if w.alive and w.wid not in self._suspect)

    def _regroup_step(self) -> bool:
        """Start a regroup epoch once the future members are idle: every live worker (rank 0
        first, then by worker id) except one parked on an abandoned assignment (hung) or
        that never answered the last regroup.  Returns True while the dispatcher must hold
        new work back (draining the members) or the epoch is running."""
        now = time.time()
        members = [w for w in sorted(self.workers.values(), key=lambda w: w.wid)
                   if w.alive and w.wid not in self._suspect and not (w.busy is not None and w.busy.get("abandoned"))]
        if not members or members[0].wid != 0:
            return False
        if any(self._hb_age.get(w.wid, 0.0) > 3 * HB_PERIOD_S for w in members):
            return False   # a member went quiet (dying?): keep dispatching until liveness decides
        busy = [w for w in members if w.busy is not None]
        if busy or self.coll_pending or self.coll_deferred:
            if self._regroup_drain_since is None:
                self._regroup_drain_since = now
            if now - self._regroup_drain_since < float(os.environ.get("DML_REGROUP_DRAIN_S", "120")):
                return True   # no new slices until the members are idle
            members = [w for w in members if w.busy is None]   # long slices: form without them
            if self.coll_pending or not members or members[0].wid != 0:
                return True
        self._regroup_drain_since = None
        gen = self._gen_next
        self._gen_next += 1
        # every old-generation collective thread ends at a stop appended to the task stream
        try:
            self.st.set(f"coll/{self.coll_seq}", json.dumps({"kind": "stop"}))
        except Exception:  # pragma: no cover - store gone with the service
            return False
        self.coll_seq += 1
        wids = [w.wid for w in members]
        payload = {"kind": "regroup", "gen": gen, "members": wids, "backend": self._backend,
                   "coll_base": self.coll_seq}
        self.epoch = {"kind": "regroup", "gen": gen, "members": wids, "waiting": set(wids), "ok": set(),
                      "failed": {}, "t0": now}
        log.info("re-forming the process group: generation %d over workers %s", gen, wids)
        for w in members:
            self._assign(w, payload)
        return True

    def _finish_regroup(self, ep: Dict[str, Any]) -> None:
        members = set(ep["members"])
        if not ep["failed"] and ep["ok"] == members:
            self.gen = ep["gen"]
            for w in self.workers.values():
                w.in_group = w.alive and w.wid in members
            self.dead = set()
            self.group_broken = False
            self.world = len(members)
            self.regroup_failures = 0
            self.stats["regroups"] += 1
            self.stats["generation"] = self.gen
            log.info("process group re-formed: generation %d, %d members %s (%.2fs)", self.gen, len(members),
                     sorted(members), time.time() - ep["t0"])
            return
        self.regroup_failures += 1
        self.stats["regroup_failures"] += 1
        self.group_broken = True
        for w in self.workers.values():
            if w.wid in members:
                w.in_group = False   # no member is sure to hold a usable communicator
        backoff = min(60.0, float(os.environ.get("DML_REGROUP_BACKOFF_S", "2")) * 2 ** (self.regroup_failures - 1))
        self._regroup_after = time.time() + backoff
        log.error("re-forming generation %d failed (%s); retry in %.0fs", ep["gen"], ep["failed"], backoff)
