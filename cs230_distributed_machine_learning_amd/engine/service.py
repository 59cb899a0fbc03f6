"""Controller: the API operations of the reference master, over the new engine.

Every route of aws-prod/master/master.py and the scheduler's
membership routes (aws-prod/scheduler/scheduler.py:95-159) is a method here returning
``(http_status, payload)``; ``gateway/app.py`` maps them onto HTTP and the client's
in-process mode (``MLTaskManager(url=None)``) calls them directly, so both paths emit
the same JSON.

Jobs are expanded into J2 subtasks (search/grid.py, engine/jobs.py), recorded in the
job table and handed to a *runner*: ``LocalRunner`` (this process, one device) or
``parallel.runner.DistributedRunner`` (one rank per GPU over RCCL).
"""
from __future__ import annotations

import glob
import os
import queue
import threading
import time
import traceback
import uuid
from typing import Any, Dict, Iterator, List, Optional, Tuple

import numpy as np

from ..config import Config
from ..data.preprocess import load_config, preprocess_frame
from ..data.registry import DatasetRegistry
from ..models.base import ParamError, family_of, is_classifier, supported_models
from ..search.grid import expand_candidates
from ..utils.log import get_logger
from ..utils import trace
from .jobs import Job, JobTable, json_safe, make_subtasks, now_iso, utc_iso
from .model_store import ModelStore
from .scheduler import Scheduler, Unit, chunk_units

log = get_logger("dml.controller")

Resp = Tuple[int, Any]


def _cv_from(cv_params: Dict[str, Any]) -> int:
    cv = cv_params.get("cv", 5)
    if cv is None:
        return 5
    if isinstance(cv, bool):
        raise ParamError("cv must be an int")
    if isinstance(cv, (int, float)):
        return int(cv)
    if isinstance(cv, str):
        digits = "".join(ch for ch in cv if ch.isdigit())
        if cv.strip().isdigit():
            return int(cv)
        if "n_splits=" in cv and digits:
            return int(cv.split("n_splits=")[1].split(",")[0].split(")")[0])
    raise ParamError(f"unsupported cv specification {cv!r} (use an int)")


def job_plan(request: Dict[str, Any]) -> Dict[str, Any]:
    """Derive everything a worker needs from a J1 request."""
    md = request.get("model_details") or {}
    model_type = md.get("model_type")
    if not model_type:
        raise ParamError("model_details.model_type is required")
    family_of(model_type)  # unsupported -> ParamError
    hp = md.get("hyperparameters") or {}
    tp = dict(request.get("train_params") or {})
    search_type = md.get("search_type")
    if search_type:
        cvp = hp.get("cv_params") or {}
        sp = hp.get("search_params") or {}
        rs = sp.get("random_state", cvp.get("random_state"))
        cands = expand_candidates(search_type, sp, random_state=rs)
        cv = _cv_from(cvp)
        scoring = cvp.get("scoring")
        error_score = cvp.get("error_score", float("nan"))
        refit = cvp.get("refit", True)
    else:
        cands = [{}]
        cv = int(tp.get("cv", 5))   # the reference always runs cross_val_score(cv=5) (worker.py:326)
        scoring = tp.get("scoring")
        error_score = float("nan")
        refit = True
    if error_score is None:
        error_score = float("nan")
    par = str(tp.get("parallelism") or "auto")
    if par not in ("auto", "task", "data"):
        raise ParamError(f"train_params.parallelism must be 'auto', 'task' or 'data', got {par!r}")
    if par == "data" and not getattr(family_of(model_type), "data_parallel", False):
        raise ParamError(f"{model_type} has no row-sharded (data-parallel) fit; use parallelism 'task'")
    return {
        "model_type": model_type, "search_type": search_type, "candidates": cands, "cv": cv,
        "scoring": scoring, "error_score": error_score, "refit": bool(refit) if not isinstance(refit, str) else True,
        "test_size": tp.get("test_size", 0.2) if tp.get("test_size") is not None else 0.2,   # D2
        "random_state": tp.get("random_state", 42) if tp.get("random_state") is not None else 42,
        "holdout": bool(tp.get("holdout", True)),
        "feature_columns": tp.get("feature_columns"), "target_column": tp.get("target_column"),
        "parallelism": par,
        # the estimator's fixed parameters (J2 merges them into every candidate): the slice
        # planner reads random_state from them (prefix_units)
        "base_params": dict(hp.get("base_estimator_params") or {}) if search_type else dict(hp),
    }


def scheduler_state_path(config: Config) -> Optional[str]:
    """Where the scheduler's learned calibration lives: next to the job journal."""
    if not config.journal:
        return None
    return os.path.join(os.path.dirname(os.path.abspath(config.journal)), "scheduler_state.json")


class Controller:
    def __init__(self, config: Optional[Config] = None, runner: Optional["Runner"] = None):
        self.config = config or Config.from_env()
        self.registry = DatasetRegistry(self.config.data_root)
        self.models = ModelStore(self.config.models_dir)
        self.table = JobTable(self.config.journal)
        self.scheduler = Scheduler(self.config.dead_after_s, self.config.algo_weight,
                                   state_path=scheduler_state_path(self.config))
        self.runner = runner or LocalRunner(self)
        if runner is not None:
            runner.bind(self)
        self._resumed = self._resume()

    def _resume(self) -> int:
        pending = self.table.replay()
        for job in pending:
            self.runner.submit(job)
        return len(pending)

    # ---- basic routes ------------------------------------------------------------------
    def home(self) -> Resp:
        return 200, {"message": "Distributed ML System API", "status": "running", "endpoints": [
            "/health", "/create_session", "/download_data/<session_id>", "/check_data/<session_id>",
            "/train/<session_id>", "/train_status/<session_id>", "/check_status/<session_id>/<job_id>",
            "/metrics/<session_id>/<job_id>", "/download_model/<session_id>/<job_id>", "/preprocess/<session_id>",
            "/workers", "/queues", "/subscribe", "/unsubscribe", "/heartbeat"],
            "models": supported_models()}

    def health(self) -> Resp:
        body = {"status": "healthy", "timestamp": time.time(), **self.table.summary(),
                "workers": len(self.scheduler.alive_workers())}
        info = getattr(self.runner, "cluster_info", None)
        if info is not None:   # the collective plane (generation, members, per-job transport)
            body["cluster"] = info()
        return 200, body

    def create_session(self) -> Resp:
        return 201, {"message": "Session created", "session_id": self.table.create_session()}

    def _bad_session(self, sid: str) -> Optional[Resp]:
        if not self.table.has_session(sid):
            return 404, {"error": "Invalid session ID"}
        return None

    # ---- data ---------------------------------------------------------------------------
    def download_data(self, sid: str, body: Dict[str, Any]) -> Resp:
        bad = self._bad_session(sid)
        if bad:
            return bad
        body = body or {}
        url, name, typ = body.get("dataset_url"), body.get("dataset_name"), body.get("dataset_type")
        if not url or not name or not typ:
            return 400, {"error": "Missing dataset parameters"}
        ok, msg = self.registry.download(url, typ, name)
        return (200, {"message": msg}) if ok else (500, {"error": msg})

    def check_data(self, sid: str, dataset_name: Optional[str]) -> Resp:
        bad = self._bad_session(sid)
        if bad:
            return bad
        if not dataset_name:
            return 400, {"error": "dataset_name is required"}
        try:
            path = self.registry.raw_file(dataset_name) or self.registry.find_file(dataset_name)
        except ValueError as e:
            return 400, {"error": str(e)}
        if path:
            return 200, {"status": f"Dataset {dataset_name} found at {path}"}
        return 404, {"error": f"Dataset {dataset_name} not found, Please Use download_data function"}

    def preprocess(self, sid: str, body: Dict[str, Any]) -> Resp:
        bad = self._bad_session(sid)
        if bad:
            return bad
        body = body or {}
        name = body.get("dataset_id")
        try:
            path = self.registry.raw_file(name) if name else None
        except ValueError as e:
            return 400, {"error": str(e)}
        if not path:
            return 404, {"error": f"Dataset {name} not found"}
        spec = body.get("yaml") or body.get("config") or body.get("yaml_url")
        if not spec:
            return 400, {"error": "Missing yaml parameters"}
        try:
            if isinstance(spec, str) and "\n" not in spec and not os.path.exists(spec):
                # reference layout: CONFIG_PATH/<dataset>/*.yaml (master.py:361-377)
                cands = sorted(glob.glob(os.path.join(self.registry.configs_dir, name, "*.yaml")))
                base = os.path.basename(spec)
                pick = [c for c in cands if os.path.basename(c) == base] or cands
                if not pick:
                    return 404, {"error": f"preprocessing config {spec!r} not found"}
                spec = pick[0]
            cfg = load_config(spec)
            import pandas as pd

            df = pd.read_csv(path)
            out = preprocess_frame(df, cfg)
            dest = self.registry.save_preprocessed(name, out)
        except Exception as e:
            return 500, {"error": f"{type(e).__name__}: {e}"}
        return 200, {"message": f"Dataset successfully preprocessed and downloaded to {os.path.dirname(dest)}",
                     "n_rows": int(len(out)), "n_cols": int(out.shape[1])}

    # ---- training -----------------------------------------------------------------------
    def _create_job(self, sid: str, body: Dict[str, Any]) -> Tuple[Optional[Job], Optional[Resp]]:
        bad = self._bad_session(sid)
        if bad:
            return None, bad
        body = dict(body or {})
        body.setdefault("job_id", str(uuid.uuid4()))
        body["session_id"] = sid
        name = body.get("dataset_id")
        try:
            path = self.registry.find_file(name) if name else None
        except ValueError as e:
            return None, (400, {"error": str(e)})
        if not path:
            return None, (404, {"error": f"Dataset {name} not found, Please Use download_data function"})
        try:
            plan = job_plan(body)
        except (ParamError, ValueError, TypeError) as e:
            return None, (400, {"error": str(e)})
        subtasks = make_subtasks(body, plan["candidates"], plan["cv"])
        try:
            job = self.table.create_job(body, subtasks, metadata=self.registry.metadata(name))   # D24
        except ValueError as e:
            return None, (409, {"error": str(e)})
        self.runner.submit(job)
        return job, None

    def train(self, sid: str, body: Dict[str, Any]) -> Resp:
        job, err = self._create_job(sid, body)
        if err:
            return err
        return 200, {"status": "Model Training Started . . . .", "job_id": job.job_id, "total_subtasks": job.total}

    def train_status(self, sid: str, body: Dict[str, Any]) -> Resp:
        """SSE stream of J7 events (master.py:209-268)."""
        job, err = self._create_job(sid, body)
        if err:
            return err

        def stream() -> Iterator[str]:
            import json

            while True:
                # read ``finished`` BEFORE the snapshot: a job finishing between the two
                # would otherwise end the stream on a non-final event
                fin = job.finished
                data = self.table.sse_json(job)
                yield f"data: {json.dumps(data)}\n\n"
                if fin:
                    break
                self.table.wait_finished(job.job_id, timeout=self.config.sse_interval_s)

        return 200, stream()

    def check_status(self, sid: str, jid: str) -> Resp:
        bad = self._bad_session(sid)
        if bad:
            return bad
        job = self.table.get(sid, jid)
        if job is None:
            return 404, {"error": f"Job {jid} not found."}
        return 200, self.table.status_json(job)

    def metrics(self, sid: str, jid: str, wait: bool = True, timeout: float = 3600.0) -> Resp:
        """J8: one J3 record per subtask; waits for the job like the reference (bounded)."""
        bad = self._bad_session(sid)
        if bad:
            return 404, {"error": "Invalid session"}
        job = self.table.get(sid, jid)
        if job is None:
            return 404, {"error": "No subtasks found"}
        if wait:
            self.table.wait_finished(jid, timeout=timeout)
        return 200, self.table.metrics_json(job)

    def download_model(self, sid: str, jid: str, body: Dict[str, Any]) -> Resp:
        bad = self._bad_session(sid)
        if bad:
            return bad
        job = self.table.get(sid, jid)
        if job is None:
            return 404, {"error": f"Job {jid} not found."}
        body = body or {}
        path = self.models.resolve(body.get("model_path"), body.get("model_id"))
        if path is None and job.result and job.result.get("best_result"):
            best = job.result["best_result"]
            path = self.models.resolve(best.get("model_path"), best.get("model_id"))
        if path is None:
            return 404, {"status": "error", "message": "Model file not found"}
        return 200, {"__file__": path, "filename": os.path.basename(path)}

    # ---- scheduler routes ------------------------------------------------------------------
    def workers(self) -> Resp:
        return 200, self.scheduler.workers_json()

    def queues(self) -> Resp:
        return 200, self.scheduler.queues()

    def subscribe(self, body: Dict[str, Any]) -> Resp:
        """Reference scheduler.py:105-117.  Under the cluster runner the answer tells the
        new worker where to join: it connects to the rendezvous store with
        ``serve --join HOST:PORT`` (``parallel/runner.py`` ``join_cluster``), gets a worker
        id from the dispatcher and starts receiving slices; the store, not this REST
        call, is its work channel.  Without a cluster runner the worker is bookkeeping
        only (single-process service)."""
        body = body or {}
        join = self.runner.join_info()
        if join is not None:
            return 200, {"status": "join", "join": join,
                         "command": f"python -m cs230_distributed_machine_learning_amd.serve --join "
                                    f"{join['host']}:{join['port']} --device {body.get('device', 'cuda:0')}"}
        wid = self.scheduler.register(body.get("host", "remote"), int(body.get("mem_capacity_mb", 0) or 0),
                                      body.get("device", "cpu"))
        return 200, {"status": "registered", "worker_id": wid}

    def unsubscribe(self, body: Dict[str, Any]) -> Resp:
        wid = str((body or {}).get("worker_id"))
        left = self.runner.leave(wid)
        units = self.scheduler.unsubscribe(wid)
        self.runner.requeue(units)
        return 200, {"status": "unsubscribed", "requeued": len(units), "left": left}

    def heartbeat(self, body: Dict[str, Any]) -> Resp:
        wid = str((body or {}).get("worker_id"))
        if not self.scheduler.heartbeat(wid):
            return 404, {"detail": "unknown worker; re-register"}
        return 200, {"status": "ok"}

    def shutdown(self) -> None:
        self.runner.shutdown()


# ======================================================================================
# runners
# ======================================================================================
class Runner:
    def bind(self, controller: Controller) -> None:
        self.ctl = controller

    def submit(self, job: Job) -> None:
        raise NotImplementedError

    def requeue(self, units: List[Unit]) -> None:
        pass

    def leave(self, worker_id: str) -> bool:
        """A worker unsubscribed: stop giving it work (runners with membership)."""
        return False

    def join_info(self) -> Optional[Dict[str, Any]]:
        """Where an extra worker joins this runner (None: no elastic membership)."""
        return None

    def shutdown(self) -> None:
        pass


class DeviceCache:
    """Resident DeviceData per (dataset file, columns, task type) on one device."""

    def _binned_only(self, ctl: Controller, plan: Dict[str, Any], X) -> bool:
        """Tree jobs on a table too large for HBM as float32 keep only its bins resident."""
        fam = family_of(plan["model_type"])
        if not str(self.device).startswith("cuda") or not (getattr(fam, "binned_ok", False)
                                                           or getattr(fam, "streams_rows", False)
                                                           or getattr(fam, "host_ok", False)):
            return False
        import torch

        free = torch.cuda.mem_get_info(torch.device(self.device))[0]
        return float(np.asarray(X).shape[0]) * np.asarray(X).shape[1] * 4 > ctl.config.stream_binned_fraction * free

    def __init__(self, device: str, max_items: int = 4):
        self.device = device
        self.max_items = max_items
        self._items: Dict[tuple, Any] = {}
        self._order: List[tuple] = []

    def get(self, ctl: Controller, plan: Dict[str, Any], dataset_id: str):
        from ..data.device import DeviceData

        ds = ctl.registry.load(dataset_id, plan["feature_columns"], plan["target_column"])
        clf = is_classifier(plan["model_type"])
        base = (ds.path, os.path.getmtime(ds.path) if ds.path else 0, tuple(ds.feature_names), ds.target_name, clf)
        # a resident float32 entry serves every job on this table (a tree job reads its bins
        # too), so the free-HBM test below never caches the same table twice; a bins-only
        # entry serves the tree jobs it was made for, and the families that stream its host rows
        full = base + (False,)
        fam = family_of(plan["model_type"])
        tree_ok = (getattr(fam, "binned_ok", False) or getattr(fam, "streams_rows", False)
                   or getattr(fam, "host_ok", False))
        for key in ((full, base + (True,)) if tree_ok else (full,)):
            if key in self._items:
                self._order.remove(key)
                self._order.append(key)
                return self._items[key]
        binned = self._binned_only(ctl, plan, ds.X)
        key = base + (binned,)
        dd = DeviceData(ds.X, ds.y, clf, self.device, name=dataset_id, binned_only=binned)
        self._items[key] = dd
        self._order.append(key)
        while len(self._order) > self.max_items:
            old = self._order.pop(0)
            self._items.pop(old, None)
        return dd


class _Sampler:
    """psutil CPU/mem sampling while a slice runs (reference worker.py:201-221), stopped in finally (D15)."""

    def __init__(self, period: float = 0.5):
        self.period = period
        self.cpu: List[float] = []
        self.mem: List[float] = []
        self._stop = threading.Event()
        self._t = None

    def __enter__(self):
        try:
            import psutil

            self._ps = psutil
            psutil.cpu_percent(None)
        except ImportError:
            self._ps = None
        self._t = threading.Thread(target=self._loop, daemon=True)
        self._t.start()
        return self

    def _loop(self):
        while not self._stop.wait(self.period):
            if self._ps:
                self.cpu.append(self._ps.cpu_percent(None))
                self.mem.append(self._ps.virtual_memory().percent)

    def __exit__(self, *a):
        self._stop.set()
        self._t.join(timeout=2)
        if self._ps and not self.cpu:
            self.cpu.append(self._ps.cpu_percent(None))
            self.mem.append(self._ps.virtual_memory().percent)

    def avg(self):
        c = float(np.mean(self.cpu)) if self.cpu else 0.0
        m = float(np.mean(self.mem)) if self.mem else 0.0
        return c, m


def candidate_costs(plan: Dict[str, Any], n_train: int, d: int, n_classes: int) -> List[float]:
    fam = family_of(plan["model_type"])
    out = []
    for c in plan["candidates"]:
        try:
            rp = fam.resolve(plan["model_type"], c, n_train, d, n_classes)
            splits = (plan["cv"] or 0) + (1 if plan["holdout"] else 0)
            out.append(fam.cost(plan["model_type"], rp, n_train, d, n_classes) * max(1, splits))
        except Exception:
            out.append(1e-3)
    return out


def run_slice(plan: Dict[str, Any], params: List[Dict[str, Any]], subtask_ids: List[str], dd, cand_ids: List[int],
              worker_id: str, device_name: str, seed: int = 0, keep_models: str = "none",
              models_root: Optional[str] = None, fault_exit: bool = False, retries: Optional[int] = None):
    """Run one slice of candidates on a device -> (results, J3 metrics per candidate, wall s).

    Controller-free so every rank of the distributed runner executes exactly this.  A
    batch that raises a transient error (injected fault, OOM) is retried up to
    ``DML_MAX_RETRIES`` times (engine/faults.py) before its candidates fail terminally.
    With ``fault_exit`` a device fault is re-raised instead: a poisoned HIP context
    cannot recover in-process, so the worker exits and the dispatcher re-queues the
    slice on a survivor.  ``retries=0`` for row-sharded slices (a one-rank retry would
    pair collectives wrongly with its peers).  ``keep_models="all"``: every candidate's
    holdout model is written to ``models_root`` and its ``model_path`` / ``model_id``
    returned in the result (reference worker.py:351-361).
    """
    from . import faults
    from .executor import CandidateResult, JobSpec, run_candidates

    keep_all = keep_models == "all" and models_root is not None and bool(plan["holdout"])
    spec = JobSpec(model_type=plan["model_type"], candidates=params, cv=plan["cv"], scoring=plan["scoring"],
                   holdout=plan["holdout"], test_size=plan["test_size"], random_state=plan["random_state"],
                   error_score=plan["error_score"], keep_models="all" if keep_all else "none", seed=seed,
                   raise_batch_errors=True)
    received = utc_iso()
    slice_key = ",".join(str(int(c)) for c in cand_ids)
    gpu = dd.device.index if dd.is_gpu else None
    if dd.is_gpu:
        import torch

        torch.cuda.reset_peak_memory_stats(dd.device)
        hbm0 = torch.cuda.memory_allocated(dd.device)
    with _Sampler() as smp:
        started = utc_iso()
        t0 = time.perf_counter()
        with trace.range(f"slice {plan['model_type']} x{len(cand_ids)}"):
            results, attempts, err = faults.run_with_retries(lambda: run_candidates(dd, spec, cand_ids), seed, slice_key,
                                                             retries=retries,
                                                             reraise=_device_fault if fault_exit else None)
        if results is None:
            results = [CandidateResult(candidate=c, ok=False, error=f"{type(err).__name__}: {err} "
                                       f"(after {attempts} attempts)") for c in cand_ids]
        wall = time.perf_counter() - t0
    finished = utc_iso()
    if keep_all:
        store = ModelStore(models_root)
        for r in results:
            if r.ok and r.model is not None:
                try:
                    r.model["subtask_id"] = subtask_ids[r.candidate]
                    r.result["model_id"] = f"{subtask_ids[r.candidate]}_model"
                    r.result["model_path"] = store.save(r.result["model_id"], r.model)
                except Exception:
                    traceback.print_exc()
                r.model = None
    cpu, mem = smp.avg()
    hbm_peak = None
    if dd.is_gpu:
        hbm_peak = int(torch.cuda.max_memory_allocated(dd.device) - hbm0)   # slice working set above resident data
    slice_fits = sum(int(r.result.get("n_fits", 0)) for r in results if r.ok)
    metrics = {}
    for r in results:
        metrics[r.candidate] = {
            "worker_id": worker_id, "subtask_id": subtask_ids[r.candidate],
            "status": "DONE" if r.ok else "FAILED", "received_at": received, "started_at": started,
            "finished_at": finished, "cpu_percent_avg": cpu, "mem_percent_avg": mem, "algo": plan["model_type"],
            "device": device_name, "fit_seconds": r.fit_seconds, "slice_wall_seconds": wall,
            "n_fits": r.result.get("n_fits", 0) if r.ok else 0, "attempts": attempts,
            # GPU fields: device index, slice HBM working set, slice throughput
            "gpu_id": gpu, "hbm_peak_bytes": hbm_peak, "slice_fits": slice_fits,
            "slice_fits_per_s": round(slice_fits / wall, 4) if wall > 0 else None,
        }
    return results, metrics, wall


def _device_fault(e: BaseException) -> bool:
    from ..parallel.runner import is_device_fault

    return is_device_fault(e)


def execute_plan_slice(ctl: Controller, job: Job, plan: Dict[str, Any], dd, cand_ids: List[int], worker_id: str,
                       device_name: str, seed: int = 0):
    params = [st.spec["parameters"] for st in job.subtasks]
    sids = [st.subtask_id for st in job.subtasks]
    return run_slice(plan, params, sids, dd, cand_ids, worker_id, device_name, seed,
                     keep_models=ctl.config.keep_models, models_root=ctl.models.root)


def presize_for_job(plan: Dict[str, Any], params: List[Dict[str, Any]], dd, slices: List[List[int]]) -> None:
    """Job setup on a worker: families with a device arena (the forest builder) size it
    once for the largest slice this job can hand the worker, so no slice pays a multi-GB
    hipMalloc mid-job."""
    fam = family_of(plan["model_type"])
    if not getattr(dd, "is_gpu", False) or not hasattr(fam, "presize") or not slices:
        return
    try:
        n_splits = (plan["cv"] or 0) + (1 if plan["holdout"] else 0)
        rps = [fam.resolve(plan["model_type"], p, int(dd.n * 0.8), dd.d, dd.n_classes) for p in params]
        # slices are re-cut once the first one calibrates the cost model: size for the
        # larger of the planned slices and a typical re-cut one (capped by the HBM budget)
        fam.presize(dd, rps, max(max(len(s) for s in slices), min(len(params), 8)), max(1, n_splits))
    except Exception:
        traceback.print_exc()


def prefix_units(plan: Dict[str, Any], todo: List[int]) -> List[List[int]]:
    """Candidates that one device batch can grow as ONE ensemble (models/base.py
    ``prefix_groups``: forests / boosting differing only in n_estimators, with a fixed
    random_state, no early stopping) form one scheduling unit, so a slice never splits a group
    and its cost is the longest member's; every other candidate is a unit of its own."""
    import os

    mt = plan["model_type"]
    if not (mt.startswith("RandomForest") or mt.startswith("GradientBoosting")) or \
            os.environ.get("DML_PREFIX_SHARE", "1") == "0":
        return [[i] for i in todo]
    units: Dict[Any, List[int]] = {}
    for i in todo:
        c = {**(plan.get("base_params") or {}), **plan["candidates"][i]}
        if c.get("random_state") in (None, "None") or c.get("n_iter_no_change") not in (None, "None"):
            key: Any = ("solo", i)
        else:
            # forests also nest max_depth (prefix_groups depth=True) unless pruning / monotonic
            # clipping rewrites the grown trees
            drop = {"n_estimators"}
            if mt.startswith("RandomForest") and not c.get("max_leaf_nodes") and not c.get("ccp_alpha") and \
                    c.get("monotonic_cst") is None:
                drop.add("max_depth")
            key = repr(sorted((k, repr(v)) for k, v in c.items() if k not in drop))
        units.setdefault(key, []).append(i)
    return list(units.values())


def plan_slices(ctl: Controller, plan: Dict[str, Any], todo: List[int], n_train: int, d: int, n_classes: int,
                min_slices: int = 1) -> List[List[int]]:
    """LPT order (most expensive first) cut into ~chunk_target_s slices, over scheduling units
    (``prefix_units``: a prefix-sharing group is priced at its longest member)."""
    costs = candidate_costs(plan, n_train, d, n_classes)
    units = prefix_units(plan, todo)
    ucost = [max(costs[i] for i in u) for u in units]
    order = sorted(range(len(units)), key=lambda k: -ucost[k])
    est = [ctl.scheduler.estimate(plan["model_type"], ucost[k]) for k in order]
    chunk_ids = chunk_units(est, ctl.config.chunk_target_s, min_slices)
    slices: Dict[int, List[int]] = {}
    for k, c in zip(order, chunk_ids):
        slices.setdefault(int(c), []).extend(units[k])
    return [slices[k] for k in sorted(slices)]


def should_recut(ctl: Controller, plan: Dict[str, Any], queued: List[List[int]], costs: List[float]) -> bool:
    """True when the queued slices, priced with the CURRENT calibration, are far from
    ``chunk_target_s``: the median is under half the target, or over twice it while some
    slice still holds several candidates.  A job is cut with the prior seconds-per-cost
    and the first slices (cold caches, lazy device copies) can mis-calibrate it; slices of
    one candidate leave most of the GPU idle at the top tree levels."""
    if len(queued) < 2:
        return False
    T = ctl.config.chunk_target_s
    if T <= 0:
        return False
    est = sorted(ctl.scheduler.estimate(plan["model_type"], sum(costs[c] for c in sl)) for sl in queued)
    med = est[len(est) // 2]
    return med < 0.5 * T or (med > 2.0 * T and any(len(sl) > 1 for sl in queued))


def publish_results(ctl: Controller, job: Job, results, metrics) -> None:
    for r in results:
        st = job.subtasks[r.candidate]
        ok = r.ok if hasattr(r, "ok") else r["ok"]
        if ok:
            R = dict(r.result if hasattr(r, "result") else r["result"])
            R.setdefault("model_id", f"{st.subtask_id}_model")
            R.setdefault("model_path", None)
            ctl.table.finish_subtask(job.job_id, st.subtask_id, "completed", result=json_safe(R),
                                     metrics=metrics.get(r.candidate))
        else:
            ctl.table.finish_subtask(job.job_id, st.subtask_id, "failed",
                                     error=r.error if hasattr(r, "error") else r.get("error"),
                                     metrics=metrics.get(r.candidate))


def refit_model(plan: Dict[str, Any], params: Dict[str, Any], dd) -> Optional[Dict[str, Any]]:
    """Fit one candidate on every row.  Under a RowShard every rank calls this in lock
    step (the fit's reductions are collectives); only rank 0 keeps the model."""
    from ..search.cv import ROLE_TRAIN
    from .executor import JobSpec, build_tasks

    spec = JobSpec(model_type=plan["model_type"], candidates=[params], cv=0, holdout=False, keep_models="all",
                   scoring=plan["scoring"])
    # a single "full" split: train on every row; the executor scores nothing
    roles = np.full((1, getattr(dd, "n_global", dd.n)), ROLE_TRAIN, dtype=np.uint8)
    dd.set_splits(roles, ["full"], key=("full",))
    fam = family_of(plan["model_type"])
    tasks, errors = build_tasks(dd, spec, [0])
    if errors or not tasks:
        return None
    outs = fam.run(dd, tasks, keep_models=True)
    if not outs or outs[0].model is None:
        return None
    return outs[0].model


def refit_best(ctl: Controller, job: Job, plan: Dict[str, Any], dd, best_idx: int) -> Optional[str]:
    """sklearn refit=True: fit the best candidate on all rows and store the artefact."""
    from .executor import JobSpec, run_candidates

    model = refit_model(plan, job.subtasks[best_idx].spec["parameters"], dd)
    if model is None:
        return None
    model["job_id"] = job.job_id
    model["subtask_id"] = job.subtasks[best_idx].subtask_id
    model["feature_names"] = list(ctl.registry.load(job.dataset_id, plan["feature_columns"],
                                                    plan["target_column"]).feature_names)
    return ctl.models.save(f"{job.subtasks[best_idx].subtask_id}_model", model)


class _JobRun:
    """A job in flight on the local runner: its remaining LPT slices and partial results."""

    def __init__(self, job: Job, plan: Dict[str, Any], dd, slices: List[List[int]], costs: List[float], seq: int):
        self.job, self.plan, self.dd, self.costs, self.seq = job, plan, dd, costs, seq
        self.slices = list(slices)
        self.si = 0
        self.rechunked = False
        self.recuts = 0
        self.results: List[Any] = []


class LocalRunner(Runner):
    """Runs jobs in this process on one device (``Config.device``) with session fair share.

    Candidates of a job are ordered LPT (most expensive first) and cut into slices of about
    ``chunk_target_s`` estimated seconds.  Between slices the runner picks the active job
    of the session that has used the least device time so far (ties: arrival order), so a
    small job submitted behind a large search finishes in seconds instead of waiting for
    it (reference: one Kafka FIFO for all sessions).  Status/SSE progress
    streams slice by slice while the device stays batched within each slice.
    """

    def __init__(self, controller: Optional[Controller] = None):
        self.q: "queue.Queue[Optional[Job]]" = queue.Queue()
        self._thread: Optional[threading.Thread] = None
        self.cache: Optional[DeviceCache] = None
        self.session_used: Dict[str, float] = {}
        self._seq = 0
        if controller is not None:
            self.bind(controller)

    def bind(self, controller: Controller) -> None:
        super().bind(controller)
        self.device = controller.config.resolved_device()
        self.cache = DeviceCache(self.device)
        self.worker_id = controller.scheduler.register("local", 0, self.device)
        self._hb_stop = threading.Event()

    def submit(self, job: Job) -> None:
        if self._thread is None:
            self._thread = threading.Thread(target=self._loop, name="dml-local-runner", daemon=True)
            self._thread.start()
        self.q.put(job)

    def _fail(self, job: Job, e: Exception) -> None:
        traceback.print_exc()
        for st in job.subtasks:
            if st.status not in ("completed", "failed"):
                self.ctl.table.finish_subtask(job.job_id, st.subtask_id, "failed", error=f"{type(e).__name__}: {e}")

    def _admit(self, job: Job) -> Optional[_JobRun]:
        ctl = self.ctl
        plan = job_plan(job.request)
        dd = self.cache.get(ctl, plan, job.dataset_id)
        todo = [st.index for st in job.subtasks if st.status not in ("completed", "failed")]
        if not todo:
            return None
        slices = plan_slices(ctl, plan, todo, int(dd.n * 0.8), dd.d, dd.n_classes)
        costs = candidate_costs(plan, int(dd.n * 0.8), dd.d, dd.n_classes)
        presize_for_job(plan, [st.spec["parameters"] for st in job.subtasks], dd, slices)
        self._seq += 1
        return _JobRun(job, plan, dd, slices, costs, self._seq)

    def _loop(self):
        active: List[_JobRun] = []
        stop = False
        while not stop or active:
            # admit everything submitted so far (block only when idle)
            while True:
                try:
                    job = self.q.get(block=not active and not stop)
                except queue.Empty:
                    break
                if job is None:
                    stop = True
                    if not active:
                        return
                    continue
                try:
                    jr = self._admit(job)
                    if jr is not None:
                        active.append(jr)
                        self.session_used.setdefault(job.session_id, 0.0)
                except Exception as e:  # never leave a job hanging (D5)
                    self._fail(job, e)
            if not active:
                continue
            jr = min(active, key=lambda r: (self.session_used.get(r.job.session_id, 0.0), r.seq))
            self.ctl.scheduler.heartbeat(self.worker_id)
            try:
                done = self._step(jr)
            except Exception as e:
                self._fail(jr.job, e)
                done = True
            if done:
                active.remove(jr)

    def _step(self, jr: _JobRun) -> bool:
        """Run the job's next slice; returns True when the job is complete."""
        ctl, job, plan, dd = self.ctl, jr.job, jr.plan, jr.dd
        ids = jr.slices[jr.si]
        ctl.table.mark_running(job.job_id, ids, self.worker_id)
        results, metrics, wall = execute_plan_slice(ctl, job, plan, dd, ids, self.worker_id, self.device,
                                                    seed=job_seed(job.job_id))
        self.session_used[job.session_id] = self.session_used.get(job.session_id, 0.0) + wall
        unit = Unit(unit_id=f"{job.job_id}:{jr.si}", cost=sum(jr.costs[i] for i in ids), algo=plan["model_type"])
        ctl.scheduler.observe(self.worker_id, unit, wall)
        jr.results.extend(results)
        jr.si += 1
        if jr.si < len(jr.slices) and (not jr.rechunked or should_recut(ctl, plan, jr.slices[jr.si:], jr.costs)):
            # the job was cut with the device's prior seconds-per-cost; the slices so far
            # calibrated it: re-cut the rest so slices are ~chunk_target_s of real work (a
            # GPU batch of one candidate leaves most of the chip idle at the top levels)
            jr.rechunked = True
            jr.recuts += 1
            rest = [i for sl in jr.slices[jr.si:] for i in sl]
            jr.slices = jr.slices[:jr.si] + plan_slices(ctl, plan, rest, int(dd.n * 0.8), dd.d, dd.n_classes)
        if jr.si < len(jr.slices):
            publish_results(ctl, job, results, metrics)
            return False
        # last slice: refit the winner first, so "completed" always comes with the model
        finalize_job(ctl, job, plan, dd, results)   # the earlier slices are already in the table
        publish_results(ctl, job, results, metrics)
        return True

    def run_job(self, job: Job) -> None:
        """Synchronously run one job to completion (used by tools and tests)."""
        jr = self._admit(job)
        while jr is not None and not self._step(jr):
            pass

    def shutdown(self) -> None:
        if self._thread is not None:
            self.q.put(None)


def job_seed(job_id: str) -> int:
    import zlib

    return zlib.crc32(job_id.encode()) & 0xFFFF


def finalize_job(ctl: Controller, job: Job, plan: Dict[str, Any], dd, results) -> None:
    """Refit the best candidate (sklearn refit=True) and attach its model path before the
    last results are published, so "completed" always comes with the artefact."""
    best = pick_refit(ctl, job, plan, results)
    if best is None:
        return
    try:
        path = refit_best(ctl, job, plan, dd, best)
        if path:
            attach_model(ctl, job, results, best, path)
    except Exception:
        traceback.print_exc()


def pick_refit(ctl: Controller, job: Job, plan: Dict[str, Any], results) -> Optional[int]:
    """Index of the candidate to refit on all rows -- the job's best by mean CV score over
    every result so far (already published subtasks + ``results``), ties to the lowest
    index like jobs.aggregate_best -- or None (refit=False, keep_models='none', no success)."""
    if not plan.get("refit", True) or ctl.config.keep_models == "none":
        return None
    pool: Dict[int, float] = {}
    for st in job.subtasks:
        if st.status == "completed" and st.result:
            pool[st.index] = score_r(st.result)
    for r in results:
        if r.ok:
            pool[r.candidate] = score_r(r.result)
    if not pool:
        return None
    return max(pool, key=lambda i: (pool[i], -i))


def attach_model(ctl: Controller, job: Job, results, cand: int, path: str) -> None:
    """The refit model's path goes on the winner's J4 result: in the not-yet-published
    ``results`` when it is there, else on its already-published subtask."""
    for r in results:
        if r.candidate == cand and r.ok:
            r.result["model_path"] = path
            return
    ctl.table.attach_model(job.job_id, job.subtasks[cand].subtask_id, path)


def score_r(R: Dict[str, Any]) -> float:
    v = R.get("mean_cv_score")
    return -np.inf if v is None or (isinstance(v, float) and np.isnan(v)) else v
