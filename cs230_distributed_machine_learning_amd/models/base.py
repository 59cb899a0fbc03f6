"""Estimator families: typed registry + the batched-fit interface.

The reference instantiates estimators with ``exec``/``eval`` of
``"{name}(**{parameters})"`` over a 15-name whitelist
(aws-prod/worker/worker.py:36-57, :436-455; defect D19).  Here every supported name
maps to a *family* object that (a) validates and resolves the sklearn-style parameter
dict into numeric settings, (b) prices a fit for the scheduler, and (c) runs MANY fits
(candidates x CV folds x holdout) in one batched device call.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence


class ParamError(ValueError):
    """Invalid estimator parameter (reported as a failed subtask, never a crash)."""


@dataclass
class FitTask:
    task_id: int
    candidate: int
    split: int
    model_type: str
    params: Dict[str, Any]
    seed: int = 0
    keep: bool = True           # with keep_models: this fit's model is wanted (holdout fits only, when there is one)
    need_proba: bool = False    # the job's scorer reads class probabilities (roc_auc, neg_log_loss, ...)


@dataclass
class FitOutput:
    task_id: int
    pred: Any = None            # device tensor aligned with the split's test rows
    proba: Any = None           # optional [n_test, C]
    decision: Any = None        # optional binary decision_function [n_test] (SVC: roc_auc / average_precision)
    fit_seconds: float = 0.0    # amortised device time of this fit
    error: Optional[str] = None
    model: Any = None           # optional fitted model (when asked to keep it)
    info: Dict[str, Any] = field(default_factory=dict)


class Family:
    model_types: Sequence[str] = ()
    classifiers: Sequence[str] = ()

    def is_classifier(self, model_type: str) -> bool:
        return model_type in self.classifiers

    def resolve(self, model_type: str, params: Dict[str, Any], n_train: int, n_features: int,
                n_classes: int) -> Dict[str, Any]:
        raise NotImplementedError

    def cost(self, model_type: str, rp: Dict[str, Any], n_train: int, n_features: int, n_classes: int) -> float:
        return 1.0

    def run(self, data, tasks: List[FitTask], keep_models: bool = False) -> List[FitOutput]:
        raise NotImplementedError


_REGISTRY: Dict[str, Family] = {}


def register(family: Family) -> Family:
    for name in family.model_types:
        _REGISTRY[name] = family
    return family


def family_of(model_type: str) -> Family:
    _ensure_loaded()
    try:
        return _REGISTRY[model_type]
    except KeyError:
        raise ParamError(f"Unsupported model: {model_type}") from None


def supported_models() -> List[str]:
    _ensure_loaded()
    return sorted(_REGISTRY)


def is_classifier(model_type: str) -> bool:
    return family_of(model_type).is_classifier(model_type)


_loaded = False


def _ensure_loaded():
    global _loaded
    if _loaded:
        return
    _loaded = True
    from . import forest, linear, neighbors, boosting, svm, transformers  # noqa: F401


# ---- common parameter helpers ---------------------------------------------------------
def as_bool(v, name):
    if isinstance(v, bool):
        return v
    if isinstance(v, (int,)) and v in (0, 1):
        return bool(v)
    if isinstance(v, str) and v.lower() in ("true", "false"):
        return v.lower() == "true"
    raise ParamError(f"{name} must be a bool, got {v!r}")


def as_int(v, name, lo=None, hi=None, allow_none=False):
    if v is None and allow_none:
        return None
    if isinstance(v, bool) or not isinstance(v, (int, float)) or (isinstance(v, float) and not v.is_integer()):
        if isinstance(v, str):
            try:
                v = int(v)
            except ValueError:
                raise ParamError(f"{name} must be an int, got {v!r}") from None
        else:
            raise ParamError(f"{name} must be an int, got {v!r}")
    v = int(v)
    if lo is not None and v < lo:
        raise ParamError(f"{name} must be >= {lo}, got {v}")
    if hi is not None and v > hi:
        raise ParamError(f"{name} must be <= {hi}, got {v}")
    return v


def as_float(v, name, lo=None, hi=None, allow_none=False):
    if v is None and allow_none:
        return None
    if isinstance(v, bool):
        raise ParamError(f"{name} must be a float, got {v!r}")
    try:
        v = float(v)
    except (TypeError, ValueError):
        raise ParamError(f"{name} must be a float, got {v!r}") from None
    if math.isnan(v):
        raise ParamError(f"{name} must not be NaN")
    if lo is not None and v < lo:
        raise ParamError(f"{name} must be >= {lo}, got {v}")
    if hi is not None and v > hi:
        raise ParamError(f"{name} must be <= {hi}, got {v}")
    return v


def prefix_groups(tasks: Sequence[FitTask], ok=None, depth: bool = False):
    """Exact sharing of ensemble prefixes inside one batch of fits.

    Fits that differ only in ``n_estimators``, on the same split, with an explicit
    ``random_state``, grow the SAME first trees / stages: tree j's seed depends only on the
    random state and j (forest.py ``native_seed``; boosting draws its subsamples and feature
    orders from the same seeded generators stage by stage), exactly as sklearn's estimators
    with a fixed random_state do.  Only the longest fit of such a group (the leader) is
    grown; every shorter one (a follower) is scored from the leader's first n_estimators
    trees / stages -- the same model, bit for bit, as growing it alone.  ``depth=True``
    (forests on the GPU predictor) also nests ``max_depth``: a tree grown to depth D holds the
    tree grown to d < D as its top d levels (same node-keyed feature orders, same splits; a
    node at depth d is that tree's leaf, with its stored class sums), so one leader with the
    most trees AND the deepest trees serves every (n_estimators, max_depth) of its group --
    unless pruning (max_leaf_nodes, ccp_alpha) or monotonic clipping rewrite the grown trees.
    ``ok(task)`` excludes fits whose later stages change earlier results (early stopping).
    DML_PREFIX_SHARE=0 turns the sharing off.  Returns (leaders in input order,
    {leader task_id: followers}).  The reference grows every candidate separately
    (aws-prod/worker/worker.py:315-341)."""
    import os

    if os.environ.get("DML_PREFIX_SHARE", "1") == "0":
        return list(tasks), {}

    def nested_depth(t: FitTask) -> bool:
        p = t.params
        return (depth and "max_depth" in p and not p.get("max_leaf_nodes") and not p.get("ccp_alpha", 0.0)
                and p.get("monotonic_cst") is None)

    def key_of(t: FitTask, drop) -> Any:
        return (t.split, t.model_type, t.need_proba,
                repr(sorted((k, repr(v)) for k, v in t.params.items() if k not in drop)))

    groups: Dict[Any, List[FitTask]] = {}
    for t in tasks:
        p = t.params
        if p.get("seed") is None or "n_estimators" not in p or (ok is not None and not ok(t)):
            key: Any = ("solo", t.task_id)
        elif nested_depth(t):
            key = ("depth",) + key_of(t, ("n_estimators", "max_depth", "warnings"))
        else:
            key = key_of(t, ("n_estimators", "warnings"))
        groups.setdefault(key, []).append(t)
    leaders, follow = [], {}

    def emit(g: List[FitTask], lead: FitTask) -> None:
        leaders.append(lead)
        rest = [t for t in g if t is not lead]
        if rest:
            follow[lead.task_id] = rest

    for key, g in groups.items():
        n_of = lambda t: t.params.get("n_estimators", 0)
        if key[0] == "depth":
            nmax = max(n_of(t) for t in g)
            dmax = max(t.params["max_depth"] for t in g)
            lead = next((t for t in g if n_of(t) == nmax and t.params["max_depth"] == dmax), None)
            if lead is not None:
                emit(g, lead)
                continue
            subs: Dict[Any, List[FitTask]] = {}   # no dominating fit: share n_estimators only
            for t in g:
                subs.setdefault(t.params["max_depth"], []).append(t)
            for sg in subs.values():
                emit(sg, max(sg, key=n_of))
            continue
        emit(g, max(g, key=n_of))
    order = {t.task_id: i for i, t in enumerate(tasks)}
    leaders.sort(key=lambda t: order[t.task_id])
    return leaders, follow


def seed_of(random_state) -> Optional[int]:
    """random_state on the wire: int, None, or a str(RandomState) -> None."""
    if random_state is None:
        return None
    if isinstance(random_state, bool):
        return int(random_state)
    if isinstance(random_state, (int,)):
        return int(random_state) & 0xFFFFFFFFFFFF
    if isinstance(random_state, float) and random_state.is_integer():
        return int(random_state)
    if isinstance(random_state, str):
        try:
            return int(random_state)
        except ValueError:
            return None
    return None


IGNORED_COMMON = {"n_jobs", "verbose", "warm_start", "copy_X", "positive_ignored"}
