"""Job table: sessions -> jobs -> subtasks, result aggregation, JSON contract, journal.

Replaces the reference's Redis keyspace (aws-prod/master/redis_util.py:20-169,
SURVEY §2.4) and result collector (aws-prod/master/task_handler.py:18-123,254-263)
with an in-memory, lock-protected table owned by the controller:

* per-job counters instead of ``KEYS`` scans (D17) and one table instead of one
  never-ending Kafka consumer thread per job (D16);
* terminal states ``completed`` AND ``failed`` both count toward completion (D5); the
  best candidate is chosen among successful ones by ``mean_cv_score`` (J5);
* ``tasks_pending`` is computed from the table (D25);
* an append-only JSONL journal (``--journal``) records job specs and terminal subtask
  results; ``JobTable.replay`` rebuilds the table after a restart and reports the
  non-terminal subtasks to re-enqueue.

JSON shapes produced here: J2 subtask, J5 final result, J6 status, J7
SSE event, J8 metrics list.
"""
from __future__ import annotations

import json
import math
import os
import threading
import time
import uuid
from dataclasses import dataclass, field
from datetime import datetime, timezone
from typing import Any, Dict, Iterable, List, Optional


def now_iso() -> str:
    return datetime.now().isoformat()


def utc_iso() -> str:
    return datetime.now(timezone.utc).isoformat() + "Z"


def json_safe(obj: Any) -> Any:
    """NaN/Inf -> None recursively (the client's _clean_dict rule, core.py:72-80)."""
    if isinstance(obj, float):
        return None if (math.isnan(obj) or math.isinf(obj)) else obj
    if isinstance(obj, dict):
        return {k: json_safe(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [json_safe(v) for v in obj]
    try:
        import numpy as np

        if isinstance(obj, np.generic):
            return json_safe(obj.item())
        if isinstance(obj, np.ndarray):
            return json_safe(obj.tolist())
    except ImportError:  # pragma: no cover
        pass
    return obj


TERMINAL = ("completed", "failed")


@dataclass
class Subtask:
    subtask_id: str
    index: int
    spec: Dict[str, Any]                 # J2
    status: str = "pending"              # pending | running | completed | failed
    result: Optional[Dict[str, Any]] = None
    error: Optional[str] = None
    completed_at: Optional[str] = None
    worker: Optional[str] = None
    attempts: int = 0
    metrics: Optional[Dict[str, Any]] = None   # J3


@dataclass
class Job:
    job_id: str
    session_id: str
    dataset_id: str
    model_type: str
    search_type: Optional[str]
    request: Dict[str, Any]
    subtasks: List[Subtask]
    created_at: str = field(default_factory=now_iso)
    metadata: Dict[str, Any] = field(default_factory=dict)
    n_done: int = 0
    n_failed: int = 0
    result: Optional[Dict[str, Any]] = None
    finished: bool = False
    started_ts: float = field(default_factory=time.time)
    finished_ts: Optional[float] = None
    error: Optional[str] = None
    fits_done: int = 0                   # CV/holdout fits of completed subtasks (north-star counter)

    def fits_per_s(self) -> float:
        dt = (self.finished_ts or time.time()) - self.started_ts
        return self.fits_done / dt if dt > 0 else 0.0

    @property
    def total(self) -> int:
        return len(self.subtasks)

    @property
    def status(self) -> str:
        if self.finished:
            return "failed" if (self.n_done == 0 and self.total > 0) else "completed"
        if self.n_done + self.n_failed == 0:
            return "pending"
        return str(100.0 * (self.n_done + self.n_failed) / max(1, self.total))


class JobTable:
    def __init__(self, journal_path: Optional[str] = None):
        self._lock = threading.RLock()
        self._cond = threading.Condition(self._lock)
        self.sessions: Dict[str, float] = {}
        self.jobs: Dict[str, Job] = {}
        self.journal_path = journal_path
        self._journal = None
        self.node_fits = 0                    # fits completed by this controller since start
        self.node_t0 = time.time()
        if journal_path:
            os.makedirs(os.path.dirname(os.path.abspath(journal_path)), exist_ok=True)

    # ---- journal ---------------------------------------------------------------------
    def _log(self, event: Dict[str, Any]) -> None:
        if not self.journal_path:
            return
        if self._journal is None:
            self._journal = open(self.journal_path, "a", encoding="utf-8")
        self._journal.write(json.dumps(json_safe(event)) + "\n")
        self._journal.flush()

    def replay(self) -> List[Job]:
        """Rebuild from the journal; returns jobs with non-terminal subtasks."""
        if not self.journal_path or not os.path.exists(self.journal_path):
            return []
        with self._lock:
            with open(self.journal_path, "r", encoding="utf-8") as f:
                for line in f:
                    line = line.strip()
                    if not line:
                        continue
                    try:
                        ev = json.loads(line)
                    except json.JSONDecodeError:
                        continue  # torn last line after a crash
                    kind = ev.get("event")
                    if kind == "session":
                        self.sessions[ev["session_id"]] = ev.get("ts", time.time())
                    elif kind == "job":
                        self._create_job(ev["request"], ev["subtasks"], ev.get("metadata", {}), log=False)
                    elif kind == "subtask":
                        job = self.jobs.get(ev["job_id"])
                        if job:
                            self._finish_subtask(job, ev["subtask_id"], ev["status"], ev.get("result"),
                                                 ev.get("error"), ev.get("metrics"), log=False)
                    elif kind == "result_update":
                        job = self.jobs.get(ev["job_id"])
                        idx = _subtask_index(ev["subtask_id"])
                        if job and idx is not None and idx < job.total and job.subtasks[idx].result is not None:
                            job.subtasks[idx].result = dict(job.subtasks[idx].result, **ev.get("fields", {}))
                    elif kind == "model":
                        job = self.jobs.get(ev["job_id"])
                        idx = _subtask_index(ev["subtask_id"])
                        if job and idx is not None and idx < job.total and job.subtasks[idx].result is not None:
                            job.subtasks[idx].result = dict(job.subtasks[idx].result, model_path=ev["model_path"])
                            if job.finished:
                                self._complete(job)
            return [j for j in self.jobs.values() if not j.finished]

    # ---- sessions ----------------------------------------------------------------------
    def create_session(self) -> str:
        sid = str(uuid.uuid4())
        with self._lock:
            self.sessions[sid] = time.time()
            self._log({"event": "session", "session_id": sid, "ts": time.time()})
        return sid

    def has_session(self, sid: str) -> bool:
        with self._lock:
            return sid in self.sessions

    # ---- jobs ----------------------------------------------------------------------------
    def create_job(self, request: Dict[str, Any], subtasks: List[Dict[str, Any]], metadata=None) -> Job:
        with self._lock:
            return self._create_job(request, subtasks, metadata or {}, log=True)

    def _create_job(self, request, subtasks, metadata, log: bool) -> Job:
        md = request.get("model_details", {})
        job = Job(
            job_id=request["job_id"], session_id=request["session_id"], dataset_id=request.get("dataset_id", ""),
            model_type=md.get("model_type", ""), search_type=md.get("search_type"), request=request,
            subtasks=[Subtask(subtask_id=s["subtask_id"], index=i, spec=s) for i, s in enumerate(subtasks)],
            metadata=dict(metadata),
        )
        if job.job_id in self.jobs:
            raise ValueError(f"job {job.job_id} already exists")
        self.jobs[job.job_id] = job
        self.sessions.setdefault(job.session_id, time.time())
        if log:
            self._log({"event": "job", "request": request, "subtasks": subtasks, "metadata": metadata})
        if not job.subtasks:
            self._complete(job)
        return job

    def get(self, session_id: str, job_id: str) -> Optional[Job]:
        with self._lock:
            job = self.jobs.get(job_id)
            if job is None or job.session_id != session_id:
                return None
            return job

    def mark_running(self, job_id: str, indices: Iterable[int], worker: str) -> None:
        with self._lock:
            job = self.jobs[job_id]
            for i in indices:
                st = job.subtasks[i]
                if st.status == "pending":
                    st.status = "running"
                    st.worker = worker
                    st.attempts += 1

    def finish_subtask(self, job_id: str, subtask_id: str, status: str, result=None, error=None, metrics=None):
        with self._lock:
            job = self.jobs.get(job_id)
            if job is None:
                return
            self._finish_subtask(job, subtask_id, status, result, error, metrics, log=True)
            self._cond.notify_all()

    def _finish_subtask(self, job: Job, subtask_id, status, result, error, metrics, log: bool):
        idx = _subtask_index(subtask_id)
        if idx is None or idx >= job.total:
            return
        st = job.subtasks[idx]
        if st.status in TERMINAL:
            return  # exactly-once: duplicate results (requeue races) are ignored (D27)
        st.status = "completed" if status == "completed" else "failed"
        st.result = result
        st.error = error
        st.metrics = metrics
        st.completed_at = now_iso()
        if st.status == "completed":
            job.n_done += 1
            nf = int((result or {}).get("n_fits") or 0)
            job.fits_done += nf
            self.node_fits += nf
        else:
            job.n_failed += 1
        if log:
            self._log({"event": "subtask", "job_id": job.job_id, "subtask_id": subtask_id, "status": st.status,
                       "result": result, "error": error, "metrics": metrics})
        if job.n_done + job.n_failed == job.total:
            self._complete(job)

    def update_result(self, job_id: str, subtask_id: str, fields: Dict[str, Any]) -> None:
        """Overwrite fields of a completed subtask's result (the cluster runner's scores
        epoch replaces the progress copies with the all-gathered ones) before the job
        completes; journaled so a resumed job reads the same record."""
        with self._lock:
            job = self.jobs.get(job_id)
            if job is None:
                return
            idx = _subtask_index(subtask_id)
            if idx is None or idx >= job.total:
                return
            st = job.subtasks[idx]
            if st.result is not None:
                st.result = dict(st.result, **fields)
                self._log({"event": "result_update", "job_id": job_id, "subtask_id": subtask_id, "fields": fields})

    def attach_model(self, job_id: str, subtask_id: str, model_path: str) -> None:
        """Record the refit model's path on a completed subtask (before the job completes)."""
        with self._lock:
            job = self.jobs.get(job_id)
            if job is None:
                return
            idx = _subtask_index(subtask_id)
            if idx is None or idx >= job.total:
                return
            st = job.subtasks[idx]
            if st.result is not None:
                st.result = dict(st.result, model_path=model_path)
                self._log({"event": "model", "job_id": job_id, "subtask_id": subtask_id, "model_path": model_path})
                if job.finished and job.result is not None:
                    self._complete(job)

    def _complete(self, job: Job) -> None:
        ok = [st.result for st in job.subtasks if st.status == "completed" and st.result is not None]
        best = aggregate_best(ok)
        job.result = {"results": ok, "best_result": best, "completion_time": now_iso()}
        failed = [{"subtask_id": st.subtask_id, "error": st.error, "parameters": st.spec.get("parameters")}
                  for st in job.subtasks if st.status == "failed"]
        if failed:
            job.result["failed"] = failed
        job.finished = True
        job.finished_ts = time.time()

    def requeue_running(self, job_id: str, worker: str) -> List[int]:
        """Subtasks a lost worker held go back to pending (failure recovery)."""
        with self._lock:
            job = self.jobs.get(job_id)
            if not job:
                return []
            out = []
            for st in job.subtasks:
                if st.status == "running" and st.worker == worker:
                    st.status = "pending"
                    st.worker = None
                    out.append(st.index)
            return out

    def wait_finished(self, job_id: str, timeout: Optional[float] = None) -> bool:
        deadline = None if timeout is None else time.time() + timeout
        with self._cond:
            while True:
                job = self.jobs.get(job_id)
                if job is None or job.finished:
                    return job is not None
                rem = None if deadline is None else deadline - time.time()
                if rem is not None and rem <= 0:
                    return False
                self._cond.wait(timeout=min(1.0, rem) if rem is not None else 1.0)

    # ---- JSON views --------------------------------------------------------------------
    def status_json(self, job: Job) -> Dict[str, Any]:
        """J6 (GET /check_status) — master/master.py:146-166 shape."""
        with self._lock:
            pending = sum(1 for st in job.subtasks if st.status not in TERMINAL)
            resp = {"session_id": job.session_id, "tasks_pending": pending, "job_id": job.job_id,
                    "job_status": job.status, "total_subtasks": job.total,
                    "fits_done": job.fits_done, "fits_per_s": round(job.fits_per_s(), 4)}
            if job.finished and job.result is not None:
                resp["job_result"] = job.result
                if job.total > 1:
                    resp["best_result"] = job.result.get("best_result")
            return json_safe(resp)

    def sse_json(self, job: Job) -> Dict[str, Any]:
        """J7 — master/master.py:248-262 shape."""
        with self._lock:
            pending = sum(1 for st in job.subtasks if st.status not in TERMINAL)
            data = {"session_id": job.session_id, "job_id": job.job_id, "job_status": job.status,
                    "tasks_pending": pending, "total_subtasks": job.total,
                    "fits_done": job.fits_done, "fits_per_s": round(job.fits_per_s(), 4)}
            if job.finished and job.result is not None:
                data["job_result"] = job.result
            return json_safe(data)

    def metrics_json(self, job: Job) -> List[Dict[str, Any]]:
        """J8 — one J3 record per finished subtask."""
        with self._lock:
            return json_safe([st.metrics for st in job.subtasks if st.metrics is not None])

    def summary(self) -> Dict[str, Any]:
        with self._lock:
            return {
                "sessions": len(self.sessions),
                "jobs": len(self.jobs),
                "running": sum(1 for j in self.jobs.values() if not j.finished),
                "fits_done": self.node_fits,
                "fits_per_s_since_start": round(self.node_fits / max(1e-9, time.time() - self.node_t0), 4),
            }


def aggregate_best(results: List[Dict[str, Any]]) -> Optional[Dict[str, Any]]:
    """J5 best_result: max mean_cv_score (NaN/None sorted last) — task_handler.py:254-263."""
    if not results:
        return None

    def key(r):
        v = r.get("mean_cv_score")
        if v is None or (isinstance(v, float) and math.isnan(v)):
            return -math.inf
        return v

    return sorted(results, key=key, reverse=True)[0]


def _subtask_index(subtask_id: str) -> Optional[int]:
    try:
        return int(subtask_id.rsplit("-subtask-", 1)[1]) - 1
    except (IndexError, ValueError):
        return None


def make_subtasks(request: Dict[str, Any], candidates: List[Dict[str, Any]], cv: Optional[int]) -> List[Dict[str, Any]]:
    """J2 records in the reference's layout (task_handler.py:186-250)."""
    md = request.get("model_details", {})
    job_id, sid = request["job_id"], request["session_id"]
    train_params = dict(request.get("train_params") or {})
    is_search = "search_type" in md
    hp = md.get("hyperparameters", {}) or {}
    base = hp.get("base_estimator_params", {}) if is_search else hp
    out = []
    for i, cand in enumerate(candidates):
        params = {**base, **cand}
        tp = {"cv": cv, **train_params} if is_search else dict(train_params)
        out.append({
            "subtask_id": f"{job_id}-subtask-{i + 1}", "job_id": job_id, "session_id": sid,
            "dataset_id": request.get("dataset_id"), "model_type": md.get("model_type"),
            "parameters": params, "train_params": tp,
        })
    return out
