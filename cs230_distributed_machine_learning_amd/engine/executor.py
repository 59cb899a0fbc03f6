"""Fit executor: turns a job's candidates into device-batched fit tasks and results.

This is the MI355X replacement for the reference worker's per-task hot path
(aws-prod/worker/worker.py:289-363 ``train_model``): one ``fit`` on a holdout split +
``cross_val_score(cv=5)`` per candidate, each re-reading the CSV.  Here:

1. splits (CV folds + holdout) become one role tensor on the device (search/cv.py);
2. every (candidate, split) becomes a ``FitTask`` with resolved parameters;
3. tasks are grouped by estimator family and run in as few device batches as memory
   allows (models/*.py);
4. predictions are scored on-device (search/scoring.py) and folded into the
   reference's per-candidate result dict (J4 ``R``), with the intended semantics of
   defects D1/D2/D5/D6 (holdout actually works, cv/scoring honoured, failures terminal).

``run_candidates`` is what a worker rank executes for the candidate slice the
scheduler assigned to it.
"""
from __future__ import annotations

import math
import time
import traceback
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

from ..models.base import FitOutput, FitTask, ParamError, family_of, is_classifier
from ..search import scoring as scoring_mod
from ..utils import trace
from ..search.cv import make_split_roles


@dataclass
class JobSpec:
    """Everything a worker needs to run a job's fits (derived from J1/J2)."""

    model_type: str
    candidates: List[Dict[str, Any]]          # full estimator params per candidate (base + point)
    cv: int = 5
    scoring: Optional[str] = None
    holdout: bool = True
    test_size: Any = 0.2
    random_state: Any = 42
    error_score: Any = float("nan")
    return_train_score: bool = False
    keep_models: str = "best"                 # none | best | all
    seed: int = 0
    raise_batch_errors: bool = False          # device errors propagate (the caller retries the batch)

    def split_key(self):
        return (self.cv, self.holdout, str(self.test_size), str(self.random_state), is_classifier(self.model_type))


@dataclass
class CandidateResult:
    candidate: int
    ok: bool
    result: Dict[str, Any] = field(default_factory=dict)   # J4 R
    error: Optional[str] = None
    model: Any = None
    fit_seconds: float = 0.0


def prepare_splits(data, spec: JobSpec) -> List[str]:
    key = spec.split_key()
    if key is not None and getattr(data, "_split_key", None) == key and getattr(data, "split_names", None):
        return list(data.split_names)   # the resident split roles are this job's (every slice re-asks)
    roles, names = make_split_roles(data.y_host, spec.cv if spec.cv else 0, is_classifier(spec.model_type),
                                    holdout=spec.holdout, test_size=spec.test_size,
                                    random_state=spec.random_state)
    data.set_splits(roles, names, key=spec.split_key())
    return names


def build_tasks(data, spec: JobSpec, candidate_ids: Sequence[int]):
    fam = family_of(spec.model_type)
    tasks: List[FitTask] = []
    errors: Dict[int, str] = {}
    tid = 0
    for c in candidate_ids:
        params = spec.candidates[c]
        try:
            for s in range(len(data.split_names)):
                rp = fam.resolve(spec.model_type, params, data.train_counts[s], data.d, data.n_classes)
                tasks.append(FitTask(task_id=tid, candidate=c, split=s, model_type=spec.model_type, params=rp,
                                     seed=(spec.seed * 1000003 + c) & 0xFFFFFFFF))
                tid += 1
        except (ParamError, ValueError, TypeError) as e:
            errors[c] = f"{type(e).__name__}: {e}"
            tasks = [t for t in tasks if t.candidate != c]
    return tasks, errors


def _batched_scores(data, tasks, outputs: Dict[int, FitOutput], scorer: str) -> Dict[int, float]:
    """Accuracy of every device fit in a few launches and ONE device->host read: fits are
    grouped by split (same held-out rows), their predictions stacked and scored together --
    instead of one reduction and one host sync per fit (a 2,560-fit LogisticRegression batch
    spent 0.27 s per search in per-fit syncs).  Exact: a mean of 0/1 counts is the same
    double whatever the reduction order (so only accuracy is batched here)."""
    if scorer != "accuracy" or not getattr(data, "is_gpu", False):
        return {}
    by_split: Dict[int, List[FitTask]] = {}
    for t in tasks:
        o = outputs.get(t.task_id)
        if o is None or o.error or not isinstance(o.pred, torch.Tensor) or not o.pred.is_cuda:
            continue
        by_split.setdefault(t.split, []).append(t)
    ids, vals = [], []
    for sp, ts in by_split.items():
        y = data.test_targets(sp)
        if y.numel() == 0 or any(outputs[t.task_id].pred.numel() != y.numel() for t in ts):
            continue
        P = torch.stack([outputs[t.task_id].pred.reshape(-1) for t in ts])
        vals.append((P.long() == y.long().view(1, -1)).double().mean(1))
        ids.extend(t.task_id for t in ts)
    if not vals:
        return {}
    return dict(zip(ids, torch.cat(vals).cpu().tolist()))


def _scores_for(data, task: FitTask, out: FitOutput, scorer: str, pre: Optional[Dict[int, float]] = None):
    if pre is not None and task.task_id in pre:
        return pre[task.task_id]
    if scorer == "score":
        return float(out.info["score"])
    y = data.test_targets(task.split)
    return scoring_mod.score(scorer, y, out.pred, data.n_classes, out.proba, decision=out.decision)


def run_candidates(data, spec: JobSpec, candidate_ids: Sequence[int]) -> List[CandidateResult]:
    """Run every split of the given candidates; returns one result per candidate."""
    with trace.range("run_prepare"):
        names = prepare_splits(data, spec)
    clf = is_classifier(spec.model_type)
    fam = family_of(spec.model_type)
    self_scored = spec.model_type in getattr(fam, "self_scored", ())
    if self_scored:
        # estimators scored by their own ``score`` method (sklearn GridSearchCV with scoring=None)
        if spec.scoring not in (None, "None", "", "score"):
            raise ValueError(f"scoring {spec.scoring!r} needs predictions; {spec.model_type} only has score()")
        scorer = "score"
    else:
        scorer = scoring_mod.validate_scoring(spec.scoring, clf)
    if not clf and not self_scored and not getattr(data, "y_is_numeric", True):
        raise ValueError(f"{spec.model_type} needs a numeric target column; this target is categorical")
    streamable = getattr(fam, "streams_rows", False) and getattr(data, "can_stream_rows", lambda: False)()
    if getattr(data, "binned_only", False) and not getattr(fam, "binned_ok", False) and not streamable:
        if getattr(fam, "host_ok", False) and getattr(data, "can_stream_rows", lambda: False)():
            # a family with a host solver (SVC/SVR) fits on the host rows of the table, which the
            # reference also requires to fit in RAM; same splits, same scorer, CPU predictions
            data = data.host_view()
            with trace.range("run_prepare"):
                names = prepare_splits(data, spec)
        else:
            raise ValueError(f"{spec.model_type} needs the float32 rows; this table is resident only in binned "
                             f"form (too large for HBM) -- tree models only")
    sharded = getattr(data, "is_row_shard", False)
    if sharded and not getattr(fam, "data_parallel", False):
        raise ValueError(f"{spec.model_type} has no row-sharded (data-parallel) fit; run it task-parallel")
    with trace.range("run_tasks"):
        tasks, errors = build_tasks(data, spec, candidate_ids)
    if scoring_mod.needs_proba(scorer):   # families that only predict labels by default add probabilities
        for t in tasks:
            t.need_proba = True
    if data.is_gpu and not getattr(fam, "uses_forest_arena", False):
        from ..ops import forest_ops

        forest_ops.ARENA.clear(data.device)   # idle forest buffers back to the device for this family
    keep = spec.keep_models in ("all", "best")
    if keep and "holdout" in names:   # only the holdout fit's model is reported (J4 model_path)
        hold = names.index("holdout")
        for t in tasks:
            t.keep = t.split == hold
    outputs: Dict[int, FitOutput] = {}
    if tasks:
        try:
            with trace.range("run_family"):
                fam_out = fam.run(data, tasks, keep_models=keep)
            for o in fam_out:
                outputs[o.task_id] = o
            if sharded:   # rank-local held-out predictions -> the global prediction vectors
                data.gather_outputs(tasks, outputs)
        except ParamError as e:
            for t in tasks:
                errors.setdefault(t.candidate, f"ParamError: {e}")
        except Exception as e:  # device/kernel failure: every candidate of the batch fails
            if spec.raise_batch_errors:
                raise
            msg = f"{type(e).__name__}: {e}"
            for t in tasks:
                errors.setdefault(t.candidate, msg)
            traceback.print_exc()
    by_cand: Dict[int, List[FitTask]] = {}
    for t in tasks:
        by_cand.setdefault(t.candidate, []).append(t)
    cv_idx = [i for i, n in enumerate(names) if n.startswith("cv")]
    hold_idx = names.index("holdout") if "holdout" in names else None
    with trace.range("run_scores"):
        pre = _batched_scores(data, [t for t in tasks if t.split in cv_idx], outputs, scorer)
    results: List[CandidateResult] = []
    for c in candidate_ids:
        if c in errors and c not in by_cand:
            results.append(_failed(c, spec, errors[c]))
            continue
        if c in errors:
            results.append(_failed(c, spec, errors[c]))
            continue
        ts = by_cand.get(c, [])
        split_out = {t.split: (t, outputs.get(t.task_id)) for t in ts}
        cv_scores: List[float] = []
        warnings: List[str] = []
        failed_fits = 0
        for s in cv_idx:
            t, o = split_out[s]
            if o is None or o.error:
                failed_fits += 1
                if spec.error_score == "raise":
                    results.append(_failed(c, spec, o.error if o else "fit failed"))
                    break
                cv_scores.append(float(spec.error_score) if spec.error_score is not None else float("nan"))
                continue
            with trace.range("run_scores"):
                cv_scores.append(_scores_for(data, t, o, scorer, pre))
            for w in o.info.get("warnings", []):
                if w not in warnings:
                    warnings.append(w)
        else:
            R: Dict[str, Any] = {}
            fit_s = sum((split_out[s][1].fit_seconds if split_out[s][1] else 0.0) for s in split_out)
            model = None
            hold_out = split_out[hold_idx][1] if hold_idx is not None else None
            if (hold_idx is not None and (hold_out is None or hold_out.error)) or (cv_idx and failed_fits == len(cv_idx)):
                errs = [o.error for _t, o in split_out.values() if o is not None and o.error]
                results.append(_failed(c, spec, errs[0] if errs else "fit failed"))
                continue
            if hold_idx is not None:
                t, o = split_out[hold_idx]
                if self_scored:
                    R["score"] = _scores_for(data, t, o, "score")
                elif clf:
                    R["accuracy"] = _scores_for(data, t, o, "accuracy")
                else:
                    R["r2_score"] = _scores_for(data, t, o, "r2")
                    R["mean_squared_error"] = -_scores_for(data, t, o, "neg_mean_squared_error")
                R["training_time"] = o.fit_seconds
                model = o.model
            else:
                R["training_time"] = fit_s
            if cv_idx:
                R["cv_scores"] = cv_scores
                finite = [x for x in cv_scores if x is not None and not math.isnan(x)]
                R["mean_cv_score"] = float(np.mean(cv_scores)) if len(finite) == len(cv_scores) else (
                    float(np.mean(finite)) if finite and spec.error_score is None else float("nan"))
                R["std_cv_score"] = float(np.std(cv_scores)) if finite else float("nan")
            else:
                main = "score" if self_scored else ("accuracy" if clf else "r2_score")
                R["cv_scores"] = []
                R["mean_cv_score"] = R.get(main, float("nan"))
            R["scoring"] = scorer
            R["fit_time_total"] = fit_s
            its = [split_out[s][1].info.get("n_iter") for s in cv_idx if split_out[s][1] is not None]
            if its and all(i is not None for i in its):   # iterative solvers: per-fold n_iter (sklearn n_iter_)
                R["n_iter"] = [int(i) for i in its]
            R["n_fits"] = len(split_out)
            if failed_fits:
                R["failed_fits"] = failed_fits
            if warnings:
                R["warnings"] = warnings
            R["parameters"] = spec.candidates[c]
            results.append(CandidateResult(candidate=c, ok=True, result=R, model=model, fit_seconds=fit_s))
    return results


def _failed(c: int, spec: JobSpec, err: str) -> CandidateResult:
    return CandidateResult(candidate=c, ok=False, error=err, result={"parameters": spec.candidates[c]})
