"""Distributed job runner: one rank per GPU, rank 0 = controller + gateway + worker.

Replaces the reference's scheduler/worker tiers and their Kafka/HTTP plumbing
(aws-prod/scheduler/scheduler_service.py:197-351 ingress/status loops,
worker/worker.py:156-286 consume loop):

job announcement   rank 0 writes ``job/<seq>`` (the J1 request) into the TCPStore; the
                   other ranks block on that key (no spinning poll loops, D13)
dataset            rank 0 parses once; RCCL broadcast into every rank's HBM, then the
                   uint8 binned copy is derived from rank-0 edges (parallel/data.py);
                   cached per dataset for later jobs
work               candidates in LPT order (most expensive first), cut into slices;
                   every rank claims slices with ``store.add`` on one counter — dynamic
                   self-scheduling that also absorbs speed differences (work stealing)
results            per-slice result JSON through the store (rank 0 publishes progress
                   while ranks still run: streaming status/SSE), and at the end one RCCL
                   all-reduce of the [candidates x CV-folds] score matrix — the numeric
                   result path — checked against the store copy
liveness           every rank refreshes ``hb/<rank>``; rank 0's monitor re-queues the
                   claimed-but-unfinished slices of a rank that went silent, and the
                   job then finishes on the store path only (a dead rank cannot join a
                   collective)
"""
from __future__ import annotations

import json
import threading
import time
import traceback
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from ..engine import faults
from ..engine.jobs import Job, json_safe
from ..engine.service import (Controller, DeviceCache, Runner, candidate_costs, finalize_job, job_plan, job_seed,
                              plan_slices, publish_results, run_slice)
from ..models.base import family_of, is_classifier
from ..utils.log import get_logger
from . import data as pdata
from . import dist

log = get_logger("dml.runner")

HB_PERIOD_S = 1.0


class LockedStore:
    """Thread-safe view of the TCPStore for rank 0 (main loop + monitor threads).

    ``wait`` polls ``check`` so a blocked waiter never holds the lock."""

    def __init__(self, store):
        self._s = store
        self._lock = threading.Lock()

    def add(self, k, v):
        with self._lock:
            return self._s.add(k, v)

    def set(self, k, v):
        with self._lock:
            return self._s.set(k, v)

    def get(self, k):
        with self._lock:
            return self._s.get(k)

    def check(self, ks):
        with self._lock:
            return self._s.check(ks)

    def delete_key(self, k):
        with self._lock:
            return self._s.delete_key(k)

    def wait(self, ks, timeout=None):
        t0 = time.time()
        while True:
            if self.check(ks):
                return
            if timeout is not None and time.time() - t0 > timeout.total_seconds():
                raise TimeoutError(ks)
            time.sleep(0.002)


class _Res:
    """Lightweight CandidateResult rebuilt from store JSON."""

    def __init__(self, d: Dict[str, Any]):
        self.candidate = int(d["candidate"])
        self.ok = bool(d["ok"])
        self.result = d.get("result") or {}
        self.error = d.get("error")
        self.fit_seconds = float(d.get("fit_seconds", 0.0))


def _enc_results(results, metrics) -> str:
    out = []
    for r in results:
        out.append({"candidate": r.candidate, "ok": r.ok, "result": json_safe(r.result), "error": r.error,
                    "fit_seconds": r.fit_seconds, "metrics": json_safe(metrics.get(r.candidate))})
    return json.dumps(out)


class _Heartbeat:
    def __init__(self, store, rank: int):
        self.store, self.rank = store, rank
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._loop, daemon=True, name=f"dml-hb-{rank}")
        self._t.start()

    def _loop(self):
        while True:
            try:
                self.store.set(f"hb/{self.rank}", str(time.time()))
            except Exception:
                return
            if self._stop.wait(HB_PERIOD_S):
                return

    def stop(self):
        self._stop.set()


class WorkerCore:
    """What every rank does for one job (rank 0 also bookkeeps)."""

    def __init__(self, device: torch.device):
        self.inf = dist.info()
        self.store = LockedStore(dist.store())
        self.device = device
        self.cache: Dict[str, Any] = {}
        self.collectives_ok = True

    # dataset: broadcast once, keep resident
    def dataset(self, msg: Dict[str, Any], ctl: Optional[Controller]):
        from ..data.device import DeviceData

        key = msg["dataset_key"]
        if key in self.cache:
            return self.cache[key]
        plan = msg["plan"]
        X = y = None
        if self.inf.rank == 0:
            ds = ctl.registry.load(msg["dataset_id"], plan["feature_columns"], plan["target_column"])
            X, y = ds.X, ds.y
        Xd, y_host = pdata.broadcast_table(X, y, self.device)
        dd = DeviceData(Xd, y_host, is_classifier(plan["model_type"]), self.device, name=msg["dataset_id"])
        if plan["model_type"].startswith("RandomForest") or plan["model_type"].startswith("GradientBoosting"):
            pdata.share_bins(dd)
        while len(self.cache) >= 4:
            self.cache.pop(next(iter(self.cache)))
        self.cache[key] = dd
        return dd

    def dataset_dp(self, msg: Dict[str, Any], ctl: Optional[Controller]):
        """Row shard of the job's table on this rank (one RCCL scatter; parallel/data_parallel.py)."""
        from .data_parallel import RowShard, scatter_table

        key = "dp:" + msg["dataset_key"]
        if key in self.cache:
            return self.cache[key]
        plan = msg["plan"]
        X = y = None
        if self.inf.rank == 0:
            ds = ctl.registry.load(msg["dataset_id"], plan["feature_columns"], plan["target_column"])
            X, y = ds.X, ds.y
        Xs, y_glob, r0 = scatter_table(X, y, self.device)
        dd = RowShard(Xs, y_glob, r0, is_classifier(plan["model_type"]), self.device, name=msg["dataset_id"])
        while len(self.cache) >= 4:
            self.cache.pop(next(iter(self.cache)))
        self.cache[key] = dd
        return dd

    def run_dp(self, seq: int, msg: Dict[str, Any], ctl: Optional[Controller] = None):
        """Data-parallel job: every rank runs every slice in order on its row shard (the
        fits' reductions are collectives, so the ranks move in lock step); rank 0
        publishes the results, then all ranks refit the winner together."""
        from ..engine.service import refit_model

        st, r = self.store, self.inf.rank
        plan = msg["plan"]
        dd = self.dataset_dp(msg, ctl)
        params, sids = msg["params"], msg["subtask_ids"]
        for i, ids in enumerate(msg["slices"]):
            results, metrics, wall = run_slice(plan, params, sids, dd, ids, "data-parallel", str(self.device),
                                               seed=msg["seed"])
            if r == 0:
                st.set(f"job/{seq}/res/{i}", _enc_results(results, metrics))
                st.set(f"job/{seq}/wall/{i}", str(wall))
                st.add(f"job/{seq}/done", 1)
        st.add(f"job/{seq}/fin", 1)
        st.wait([f"job/{seq}/refit"])             # rank 0 picks the refit candidate (or -1)
        best = int(st.get(f"job/{seq}/refit"))
        model = refit_model(plan, params[best], dd) if best >= 0 else None
        return dd, model

    def run(self, seq: int, msg: Dict[str, Any], ctl: Optional[Controller] = None, job: Optional[Job] = None):
        if msg.get("mode") == "data":
            return self.run_dp(seq, msg, ctl)
        st, r, world = self.store, self.inf.rank, self.inf.world
        plan = msg["plan"]
        dd = self.dataset(msg, ctl)
        slices: List[List[int]] = msg["slices"]
        params, sids = msg["params"], msg["subtask_ids"]
        n_cand = len(params)
        n_cv = int(plan["cv"] or 0)
        scores = torch.zeros((n_cand, max(1, n_cv)), dtype=torch.float64, device=self.device)
        owned = torch.zeros((n_cand,), dtype=torch.float64, device=self.device)
        worker_id = f"rank{r}"
        def exec_slice(ids):
            try:
                return run_slice(plan, params, sids, dd, ids, worker_id, str(self.device), seed=msg["seed"])
            except Exception as e:  # a failing slice must not desert the job's collectives
                traceback.print_exc()
                from ..engine.executor import CandidateResult

                return [CandidateResult(candidate=c, ok=False, error=f"{type(e).__name__}: {e}") for c in ids], {}, 0.0

        def publish(i, results, metrics, wall, local):
            if local:
                for res in results:
                    if res.ok and n_cv:
                        scores[res.candidate, :n_cv] = torch.tensor(
                            [np.nan if v is None else v for v in res.result.get("cv_scores", [np.nan] * n_cv)],
                            dtype=torch.float64)
                        owned[res.candidate] = 1.0
            st.set(f"job/{seq}/res/{i}", _enc_results(results, metrics))
            st.set(f"job/{seq}/wall/{i}", str(wall))
            if st.add(f"job/{seq}/first/{i}", 1) == 1:   # count each slice once (a re-queued
                st.add(f"job/{seq}/done", 1)             # slice may finish twice)

        n_done = 0
        while True:
            i = st.add(f"job/{seq}/next", 1) - 1
            if i >= len(slices):
                break
            st.set(f"job/{seq}/claim/{i}", str(r))
            faults.maybe_kill(r, n_done)   # fault injection: die holding a claimed slice
            results, metrics, wall = exec_slice(slices[i])
            publish(i, results, metrics, wall, True)
            n_done += 1
        # Slices re-queued from a dead rank (rank 0's monitor appends them to job/<seq>/rq).
        # Stay until every slice has a result: a rank that left before the death was
        # detected would otherwise strand the re-queued work.  Each entry is claimed once.
        j = 0
        while int(st.add(f"job/{seq}/done", 0)) < len(slices):
            n_rq = int(st.add(f"job/{seq}/rq_len", 0))
            if j < n_rq:
                if st.add(f"job/{seq}/rq_claim/{j}", 1) == 1:
                    i = int(st.get(f"job/{seq}/rq/{j}"))
                    results, metrics, wall = exec_slice(slices[i])
                    publish(i, results, metrics, wall, False)   # not in this rank's RCCL share
                j += 1
                continue
            time.sleep(0.02)
        # numeric result path: one RCCL all-reduce of the score matrix (when every rank is alive)
        st.add(f"job/{seq}/fin", 1)
        st.wait([f"job/{seq}/mode"])
        mode = st.get(f"job/{seq}/mode").decode()
        if mode == "collective" and self.collectives_ok:
            dist.all_reduce_sum(scores)
            dist.all_reduce_sum(owned)
        else:
            self.collectives_ok = False
        return dd, scores, owned, mode


class DistributedRunner(Runner):
    """Rank-0 side: turns controller jobs into store announcements and publishes results."""

    def __init__(self, core: WorkerCore):
        self.core = core
        self.q: List[Job] = []
        self._cv = threading.Condition()
        self.seq = 0
        self.stop = False
        self.dead: set = set()
        self._hb_missing_since: Dict[int, float] = {}
        self.session_used: Dict[str, float] = {}

    def bind(self, controller: Controller) -> None:
        super().bind(controller)
        self.worker_ids = {}
        for r in range(dist.info().world):
            self.worker_ids[r] = controller.scheduler.register(f"rank{r}", 0, f"cuda:{r}")

    def submit(self, job: Job) -> None:
        with self._cv:
            self.q.append(job)
            self._cv.notify_all()

    def requeue(self, units) -> None:
        pass

    def shutdown(self) -> None:
        with self._cv:
            self.stop = True
            self._cv.notify_all()

    # rank 0 main loop (runs in the main thread; the gateway serves from a thread)
    def serve_forever(self, idle_poll_s: float = 0.5) -> None:
        st = self.core.store
        hb = _Heartbeat(st, 0)
        try:
            while True:
                with self._cv:
                    while not self.q and not self.stop:
                        self._cv.wait(timeout=idle_poll_s)
                    if self.stop and not self.q:
                        break
                    # session fair share at job granularity: the next job comes from the
                    # session that has used the least node time (ties: arrival order)
                    k = min(range(len(self.q)), key=lambda i: (self.session_used.get(self.q[i].session_id, 0.0), i))
                    job = self.q.pop(k)
                t_job = time.time()
                try:
                    self._run_job(job)
                except Exception as e:
                    traceback.print_exc()
                    for sub in job.subtasks:
                        if sub.status not in ("completed", "failed"):
                            self.ctl.table.finish_subtask(job.job_id, sub.subtask_id, "failed",
                                                          error=f"{type(e).__name__}: {e}")
                self.session_used[job.session_id] = self.session_used.get(job.session_id, 0.0) + time.time() - t_job
            st.set(f"job/{self.seq}", json.dumps({"shutdown": True}))
        finally:
            hb.stop()

    def _run_job(self, job: Job) -> None:
        ctl, st = self.ctl, self.core.store
        plan = job_plan(job.request)
        ds_path = ctl.registry.find_file(job.dataset_id)
        import os

        meta = ctl.registry.metadata(job.dataset_id)
        n_rows = int(meta.get("n_rows", 1000))
        todo = [sub.index for sub in job.subtasks if sub.status not in ("completed", "failed")]
        if not todo:
            return
        world = dist.info().world
        n_feat = max(1, int(meta.get("n_cols", 2)) - 1)
        data_par = self._data_parallel(plan, len(todo), n_rows, n_feat, world)
        slices = plan_slices(ctl, plan, todo, int(n_rows * 0.8), n_feat, 2,
                             min_slices=1 if data_par else min(len(todo), 2 * world))
        key = f"{ds_path}:{os.path.getmtime(ds_path)}:{plan['feature_columns']}:{plan['target_column']}:" \
              f"{is_classifier(plan['model_type'])}"
        seq = self.seq
        self.seq += 1
        msg = {"job_id": job.job_id, "dataset_id": job.dataset_id, "dataset_key": key, "plan": plan,
               "slices": slices, "params": [sub.spec["parameters"] for sub in job.subtasks],
               "subtask_ids": [sub.subtask_id for sub in job.subtasks], "seed": job_seed(job.job_id),
               "mode": "data" if data_par else "task"}
        st.set(f"job/{seq}", json.dumps(json_safe(msg)))
        for ids in slices:
            ctl.table.mark_running(job.job_id, ids, "cluster")
        if data_par:
            self._run_job_dp(job, plan, seq, msg, slices)
            return
        # progress publisher + liveness monitor while every rank (this one too) works
        done_evt = threading.Event()
        held: Dict[int, Any] = {}
        mon = threading.Thread(target=self._monitor, args=(job, seq, slices, done_evt, held), daemon=True)
        mon.start()
        dd, scores, owned, mode = self._participate(seq, msg)
        done_evt.set()
        mon.join()
        # collect everything not yet published
        results_all = []
        for i in range(len(slices)):
            raw = st.get(f"job/{seq}/res/{i}")
            for d in json.loads(raw):
                results_all.append(_Res(d))
        if mode == "collective":
            self._check_scores(results_all, scores, owned, int(plan["cv"] or 0))
        final = [held[i] for i in sorted(held)]
        finalize_job(ctl, job, plan, dd, results_all)
        for res, metrics in final:
            publish_results(ctl, job, res, metrics)
        self._cleanup(seq, len(slices))

    def _data_parallel(self, plan, n_todo: int, n_rows: int, n_feat: int, world: int) -> bool:
        """Row-sharded data parallelism (parallel/data_parallel.py) instead of task slices."""
        par = plan.get("parallelism", "auto")
        if par == "task" or world < 2 or not getattr(family_of(plan["model_type"]), "data_parallel", False):
            return False
        if par == "data":
            return True
        cfg = self.ctl.config
        cells = n_rows * n_feat
        return cells >= cfg.dp_min_cells and (n_todo < world or cells * 4 > cfg.dp_auto_gb * 2 ** 30)

    def _run_job_dp(self, job: Job, plan, seq: int, msg, slices) -> None:
        from ..engine.service import pick_refit, refit_model

        ctl, st = self.ctl, self.core.store
        done_evt = threading.Event()
        held: Dict[int, Any] = {}
        mon = threading.Thread(target=self._monitor, args=(job, seq, slices, done_evt, held), daemon=True)
        mon.start()
        # rank 0 runs the slices with everyone; the monitor publishes results as they land
        results_all = []
        refit_set, best = False, None
        try:
            dd = self.core.dataset_dp(msg, ctl)
            params, sids = msg["params"], msg["subtask_ids"]
            for i, ids in enumerate(slices):
                results, metrics, wall = run_slice(plan, params, sids, dd, ids, "data-parallel", str(self.core.device),
                                                   seed=msg["seed"])
                st.set(f"job/{seq}/claim/{i}", "0")   # the monitor's wall-time observation reads it
                st.set(f"job/{seq}/wall/{i}", str(wall))
                st.set(f"job/{seq}/res/{i}", _enc_results(results, metrics))
                st.add(f"job/{seq}/done", 1)
                results_all.extend(results)
            done_evt.set()
            mon.join()
            best = pick_refit(ctl, job, plan, results_all)
            st.set(f"job/{seq}/refit", str(best.candidate if best is not None else -1))
            refit_set = True
            if best is not None:
                try:
                    model = refit_model(plan, params[best.candidate], dd)
                    if model is not None:
                        model["job_id"] = job.job_id
                        model["subtask_id"] = job.subtasks[best.candidate].subtask_id
                        model["feature_names"] = list(ctl.registry.load(job.dataset_id, plan["feature_columns"],
                                                                        plan["target_column"]).feature_names)
                        best.result["model_path"] = ctl.models.save(f"{job.subtasks[best.candidate].subtask_id}_model",
                                                                    model)
                except Exception:
                    traceback.print_exc()
        finally:
            done_evt.set()
            if not refit_set:
                st.set(f"job/{seq}/refit", "-1")
        path = best.result.get("model_path") if refit_set and best is not None else None
        for res, metrics in [held[i] for i in sorted(held)]:
            for x in res:
                if path and x.candidate == best.candidate and x.ok:
                    x.result["model_path"] = path
            publish_results(ctl, job, res, metrics)
        self._cleanup(seq, len(slices))

    def _participate(self, seq, msg):
        # decide collective vs store-only once every live rank has finished its claims
        st = self.core.store
        t = threading.Thread(target=self._decide_mode, args=(seq,), daemon=True)
        t.start()
        out = self.core.run(seq, msg, self.ctl)
        t.join()
        return out

    def _decide_mode(self, seq):
        st = self.core.store
        world = dist.info().world
        while True:
            fin = int(st.add(f"job/{seq}/fin", 0))
            alive = world - len(self.dead)
            if fin >= alive:
                break
            time.sleep(0.05)
        st.set(f"job/{seq}/mode", "collective" if not self.dead and self.core.collectives_ok else "store")

    def _monitor(self, job: Job, seq: int, slices, done_evt: threading.Event, held: Dict[int, Any]):
        st, ctl = self.core.store, self.ctl
        published = set()
        world = dist.info().world
        last = len(slices) - 1
        while True:
            finished = done_evt.is_set()
            for i in range(len(slices)):
                if i in published:
                    continue
                try:
                    if not st.check([f"job/{seq}/res/{i}"]):
                        continue
                    raw = st.get(f"job/{seq}/res/{i}")
                except Exception:
                    continue
                items = json.loads(raw)
                res = [_Res(d) for d in items]
                metrics = {d["candidate"]: d.get("metrics") for d in items}
                published.add(i)
                if i == last:
                    held[i] = (res, metrics)   # published after the best model is refit
                else:
                    publish_results(ctl, job, res, metrics)
                try:
                    wall = float(st.get(f"job/{seq}/wall/{i}"))
                    claim = int(st.get(f"job/{seq}/claim/{i}"))
                    from ..engine.scheduler import Unit

                    ctl.scheduler.observe(self.worker_ids.get(claim, "1"),
                                          Unit(unit_id=f"{job.job_id}:{i}", cost=1.0, algo=job.model_type), wall)
                except Exception:
                    pass
            self._liveness(seq, slices, published)
            if finished and len(published) >= len(slices):
                return
            if finished:
                time.sleep(0.01)
            else:
                time.sleep(0.05)

    def _liveness(self, seq, slices, published):
        st = self.core.store
        now = time.time()
        world = dist.info().world
        for r in range(1, world):
            if r in self.dead:
                continue
            try:
                hb = float(st.get(f"hb/{r}")) if st.check([f"hb/{r}"]) else None
            except Exception:
                hb = now
            if hb is None:   # never beat: silent since we first looked
                hb = self._hb_missing_since.setdefault(r, now)
            if now - hb > self.ctl.config.dead_after_s:
                log.warning("rank %d missed heartbeats for %.1fs: re-queueing its slices", r, now - hb)
                self.dead.add(r)
                self.ctl.scheduler.unsubscribe(self.worker_ids.get(r, ""))
                for i in range(len(slices)):
                    if i in published:
                        continue
                    try:
                        if st.check([f"job/{seq}/claim/{i}"]) and int(st.get(f"job/{seq}/claim/{i}")) == r:
                            j = int(st.add(f"job/{seq}/rq_len", 1)) - 1
                            st.set(f"job/{seq}/rq/{j}", str(i))
                    except Exception:
                        pass
            else:
                self.ctl.scheduler.heartbeat(self.worker_ids.get(r, ""))
        self.ctl.scheduler.heartbeat(self.worker_ids.get(0, ""))

    @staticmethod
    def _check_scores(results, scores, owned, n_cv):
        if not n_cv:
            return
        sc = scores.cpu().numpy()
        for r in results:
            if not r.ok:
                continue
            mine = np.array([np.nan if v is None else v for v in r.result.get("cv_scores", [])], dtype=np.float64)
            if mine.size and not np.allclose(mine, sc[r.candidate, :mine.size], equal_nan=True, atol=1e-9):
                log.error("RCCL score matrix disagrees with store results for candidate %d", r.candidate)

    def _cleanup(self, seq: int, n: int) -> None:
        st = self.core.store
        for k in [f"job/{seq}"] + [f"job/{seq}/{s}/{i}" for s in ("res", "claim", "wall", "first", "rq_claim")
                                   for i in range(n)]:
            try:
                st.delete_key(k)
            except Exception:
                pass


def worker_loop(core: WorkerCore) -> None:
    """Ranks 1..N-1: wait for job announcements and run them until shutdown."""
    st = core.store
    hb = _Heartbeat(st, core.inf.rank)
    seq = 0
    try:
        while True:
            key = f"job/{seq}"
            while True:
                try:
                    st.wait([key], __import__("datetime").timedelta(seconds=60))
                    break
                except TimeoutError:
                    continue  # idle longer than the store timeout: keep waiting
                except Exception:   # the store (hosted by rank 0) is gone: the job server exited
                    log.warning("rank %d lost the controller store; leaving", core.inf.rank)
                    return
            msg = json.loads(st.get(key))
            if msg.get("shutdown"):
                return
            try:
                core.run(seq, msg, None)
            except Exception:
                traceback.print_exc()
                st.add(f"job/{seq}/fin", 1)
            seq += 1
    finally:
        hb.stop()
