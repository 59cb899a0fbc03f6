"""RandomForest{Classifier,Regressor} family — batched over candidates x splits x trees.

Parameter semantics follow sklearn's estimators the reference whitelists
(aws-prod/worker/worker.py:38,45) and fits per task (:315, :326, :341).  All trees of
all fits of a job slice are grown together by the HIP builder (ops/forest_ops.py,
csrc/kernels/forest.hip) — or by the C++ builder on CPU — in memory-budgeted batches
of whole fits, then every fit's held-out rows are predicted in one launch.

Supported: n_estimators, criterion (gini/entropy/log_loss; squared_error; friedman_mse, whose splits are
squared_error's; poisson -- sklearn's proxy sum_l log(mean_l) + sum_r log(mean_r);
absolute_error: exact weighted medians, on its own GPU builder), max_depth,
min_samples_split, min_samples_leaf (int or fraction), max_features (sqrt/log2/None/
int/float), bootstrap, max_samples, min_impurity_decrease, max_leaf_nodes (sklearn's
best-first tree: the grown tree is cut to its best-first top, ops/forest_ops.py
prune_max_leaves), random_state.  Parameters
with no effect on the fitted function (n_jobs, verbose, warm_start, oob_score) are
accepted and ignored; class_weight (dict / "balanced" / "balanced_subsample") scales
the per-class sums inside the builder exactly where sklearn's sample weights would;
ccp_alpha > 0 prunes every grown tree to its minimal cost-complexity subtree
(ops/forest_ops.py prune_ccp); min_weight_fraction_leaf bounds every side's weight
(bootstrap counts x class weights, as sklearn's sample weights) inside the builders;
monotonic_cst (regression and binary classification, sklearn's bounds and clipping) grows
on the HIP builder in every tier (per-node bounds, identical to the host builder's trees);
criterion="absolute_error" grows on the GPU MAE builder (csrc/kernels/forest_mae.hip; rows kept
in target order, exact fixed-point abs deviations) -- node for node the C++ host builder's trees,
which grow it on CPU data.
"""
from __future__ import annotations

import math
import os
import time
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from ..ops import forest_ops
from ..utils import native, trace
from .base import (Family, FitOutput, FitTask, ParamError, as_bool, as_float, as_int, prefix_groups, register,
                   seed_of)

_CLS = "RandomForestClassifier"
_REG = "RandomForestRegressor"

_DEFAULT = object()   # "parameter not given"

_DEFAULTS = {
    "n_estimators": 100, "criterion": None, "max_depth": None, "min_samples_split": 2, "min_samples_leaf": 1,
    "min_weight_fraction_leaf": 0.0, "max_features": _DEFAULT, "max_leaf_nodes": None, "min_impurity_decrease": 0.0,
    "bootstrap": True, "oob_score": False, "n_jobs": None, "random_state": None, "verbose": 0,
    "warm_start": False, "class_weight": None, "ccp_alpha": 0.0, "max_samples": None, "monotonic_cst": None,
}


def _max_features(v, d, is_cls):
    if v is _DEFAULT:        # sklearn's defaults: "sqrt" (classifier), 1.0 (regressor)
        v = "sqrt" if is_cls else 1.0
    if v is None or v == "None":   # an explicit None means every feature
        return d
    if isinstance(v, str):
        if v == "sqrt" or v == "auto":
            return max(1, int(math.sqrt(d)))
        if v == "log2":
            return max(1, int(math.log2(d)))
        raise ParamError(f"max_features {v!r} not understood")
    if isinstance(v, bool):
        raise ParamError("max_features must not be a bool")
    if isinstance(v, int) or (isinstance(v, float) and v > 1.0 and v.is_integer()):
        return max(1, min(d, int(v)))
    f = float(v)
    if not 0.0 < f <= 1.0:
        raise ParamError(f"max_features fraction must be in (0, 1], got {f}")
    return max(1, int(f * d))


def _count_param(v, n, name, lo_int):
    if isinstance(v, float):
        f = float(v)
        if not 0.0 < f <= 1.0:
            raise ParamError(f"{name} fraction must be in (0, 1], got {f}")
        return max(lo_int, int(math.ceil(f * n)))
    return as_int(v, name, lo=lo_int)


class ForestFamily(Family):
    model_types = (_CLS, _REG)
    classifiers = (_CLS,)
    uses_forest_arena = True   # batches reuse the device arena (ops/forest_ops.py ARENA)
    binned_ok = True           # fits only read the uint8 bins (DeviceData binned_only tables)
    data_parallel = True       # row-sharded fit: per-level histogram all-reduce (ops/forest_dp.py)
    dp_when_few = False        # "auto" picks the row-sharded fit for tables too large to replicate only

    def __init__(self):
        self.tiers = forest_ops.ForestTiers()
        self.hbm_budget_bytes = None  # None -> derived from free memory

    def resolve(self, model_type, params, n_train, n_features, n_classes) -> Dict[str, Any]:
        p = dict(_DEFAULTS)
        p.update({k: v for k, v in params.items() if k in _DEFAULTS})
        is_cls = model_type == _CLS
        warn: List[str] = []
        unknown = sorted(k for k in params if k not in _DEFAULTS)
        if unknown:
            warn.append(f"ignored unknown parameters {unknown}")
        crit = p["criterion"] or ("gini" if is_cls else "squared_error")
        if is_cls:
            if crit not in ("gini", "entropy", "log_loss"):
                raise ParamError(f"criterion {crit!r} invalid for {model_type}")
            crit_id = forest_ops.GINI if crit == "gini" else forest_ops.ENTROPY
        else:
            if crit not in ("squared_error", "friedman_mse", "absolute_error", "poisson"):
                raise ParamError(f"criterion {crit!r} invalid for {model_type}")
            # friedman_mse ranks splits exactly like squared_error: its proxy
            # w_l w_r (m_l - m_r)^2 is W_node x (the squared-error proxy - a node constant),
            # so the chosen splits are the same; min_impurity_decrease reads sklearn's
            # FriedmanMSE improvement (forest_common.h accept_improvement)
            crit_id = {"poisson": forest_ops.POISSON, "absolute_error": forest_ops.MAE,
                       "friedman_mse": forest_ops.FRIEDMAN}.get(crit, forest_ops.MSE)
            if crit == "poisson" and (float(p["min_impurity_decrease"] or 0.0) > 0 or float(p["ccp_alpha"] or 0.0) > 0):
                warn.append("criterion='poisson': min_impurity_decrease / ccp_alpha are applied on the "
                            "squared-error impurity scale")
        n_est = as_int(p["n_estimators"], "n_estimators", lo=1, hi=100000)
        md = as_int(p["max_depth"], "max_depth", lo=1, allow_none=True)
        mss = _count_param(p["min_samples_split"], n_train, "min_samples_split", 2)
        msl = _count_param(p["min_samples_leaf"], n_train, "min_samples_leaf", 1)
        k = _max_features(p["max_features"], n_features, is_cls)
        boot = as_bool(p["bootstrap"], "bootstrap")
        lam = 1.0
        if p["max_samples"] is not None:
            if not boot:
                raise ParamError("`max_sample` cannot be set if `bootstrap=False`")
            ms = p["max_samples"]
            if isinstance(ms, float):
                lam = float(ms)
                if not 0.0 < lam <= 1.0:
                    raise ParamError("max_samples fraction must be in (0, 1]")
            else:
                lam = min(1.0, as_int(ms, "max_samples", lo=1) / max(1, n_train))
        mid = as_float(p["min_impurity_decrease"], "min_impurity_decrease", lo=0.0)
        cw = p["class_weight"]
        if cw in ("None",):
            cw = None
        if cw is not None:
            if not is_cls:
                raise ParamError("class_weight is only valid for classifiers")
            if isinstance(cw, str):
                if cw not in ("balanced", "balanced_subsample"):
                    raise ParamError(f"class_weight {cw!r} must be a dict, 'balanced' or 'balanced_subsample'")
            elif isinstance(cw, dict):
                cw = {str(k): as_float(v, "class_weight value", lo=0.0) for k, v in cw.items()}
            else:
                raise ParamError("class_weight must be a dict, 'balanced', 'balanced_subsample' or None")
        ccp = as_float(p["ccp_alpha"], "ccp_alpha", lo=0.0)
        mln = as_int(p["max_leaf_nodes"] if p["max_leaf_nodes"] != "None" else None, "max_leaf_nodes", lo=2,
                     allow_none=True)
        mwf = as_float(p["min_weight_fraction_leaf"], "min_weight_fraction_leaf", lo=0.0, hi=0.5)
        mono = p["monotonic_cst"]
        if mono in (None, "None"):
            mono = None
        else:   # sklearn's checks and messages
            try:
                mono = [int(v) for v in mono]
            except (TypeError, ValueError):
                raise ParamError("monotonic_cst must be None or an array-like of -1, 0 or 1")
            if len(mono) != n_features:
                raise ParamError(f"monotonic_cst has shape {len(mono)} but the input data X has {n_features} features.")
            if any(v not in (-1, 0, 1) for v in mono):
                raise ParamError("monotonic_cst must be None or an array-like of -1, 0 or 1.")
            if is_cls and n_classes > 2:
                raise ParamError("Monotonicity constraints are not supported with multiclass classification")
            if crit == "absolute_error":
                warn.append("monotonic_cst with criterion='absolute_error' is not supported; ignored")
                mono = None
            elif not any(mono):
                mono = None
            elif ccp > 0 or mln:
                warn.append("monotonic_cst with ccp_alpha / max_leaf_nodes: pruning reads the clipped node values")
        return {
            "n_estimators": n_est, "criterion": crit_id, "max_depth": md if md is not None else forest_ops.INT32_MAX,
            "min_samples_split": mss, "min_samples_leaf": msl, "max_features": k, "bootstrap": int(boot),
            "lambda": lam, "min_impurity_decrease": mid, "seed": seed_of(p["random_state"]), "warnings": warn,
            "class_weight": cw, "max_leaf_nodes": mln or 0, "ccp_alpha": ccp, "min_weight_fraction_leaf": mwf,
            "monotonic_cst": mono,
        }

    def cost(self, model_type, rp, n_train, n_features, n_classes) -> float:
        """Relative device cost ~ trees x active rows x levels x features-per-node."""
        active = 0.632 * n_train * rp["lambda"] if rp["bootstrap"] else n_train
        leaves = max(1.0, active / rp["min_samples_leaf"] / max(1, rp["min_samples_split"] - 1))
        depth = min(float(rp["max_depth"]), math.log2(leaves) * 1.6 + 1)
        return rp["n_estimators"] * active * depth * rp["max_features"] * 1e-9 + 1e-3

    # ------------------------------------------------------------------------------
    def _tree_bytes(self, data, rp) -> float:
        n_train = data.n
        active = 0.632 * n_train if rp["bootstrap"] else n_train
        VC = data.n_classes if data.classification else 3
        pool = (2 * active / rp["min_samples_leaf"] + 1) * (8 + 8 * VC)
        return active * 4 * 2 + pool + active * 24

    def footprint(self, data, rp) -> tuple:
        """(active rows over the fit's trees, node-pool bound) of one fit -- the
        quantities the device workspace and node pool are sized from (forest_ops)."""
        n_train = max(data.train_counts) if getattr(data, "train_counts", None) else data.n
        if rp["bootstrap"]:
            lam = rp["lambda"]
            active = n_train * (1.0 - math.exp(-lam)) * 1.01 + 64   # Poisson(lam) weight > 0
        else:
            active = float(n_train)
        T = rp["n_estimators"]
        per_tree = 2 * active / max(1, rp["min_samples_leaf"]) + 1
        if rp["max_depth"] < 40:
            per_tree = min(per_tree, 2.0 ** (rp["max_depth"] + 1) - 1)
        return T * active, T * per_tree + T

    def _need(self, data, rows: float, T: int, pool: float) -> int:
        """Real device bytes of a batch: the builder's workspace layout + the node pool."""
        VC = data.n_classes if data.classification else 3
        return (forest_ops.workspace_bytes(int(rows), int(T), data.d, data.n_classes, not data.classification,
                                           self.tiers) + forest_ops.pool_bytes(int(pool) + 16, VC))

    def presize(self, data, rps: List[Dict[str, Any]], cands_per_batch: int, n_splits: int) -> None:
        """Grow the device arena at job setup to the largest batch this job can form, so no
        batch regrows it mid-run (a regrowth frees and maps 100+ GB: 2.6-4.7 s each,
        measured).  Workspace and node pool share one slot (ops/forest_ops.py), and every
        batch is formed under the same budget by ``_need``, so one slot of
        min(budget, the job's largest greedy batch) fits all of them.  ``rps``: resolved
        parameters per candidate; ``cands_per_batch`` is accepted for the runner's API."""
        if not data.is_gpu or not rps or getattr(data, "is_row_shard", False):
            return
        budget = self._budget(data)
        fits = []
        for rp in rps:
            rows, pool = self.footprint(data, rp)
            fits.extend([(rows, rp["n_estimators"], pool)] * max(1, n_splits))
        fits.sort(reverse=True)
        rows = pool = 0.0
        T = 0
        need = 0
        for fr, ft, fp in fits:
            nxt = self._need(data, rows + fr, T + ft, pool + fp)
            if T and nxt > budget:
                break
            rows, T, pool, need = rows + fr, T + ft, pool + fp, nxt
        need = int(min(budget, need * 1.02) + (1 << 20))    # alignment slack of the carve
        if os.environ.get("DML_ARENA_LOG"):
            import sys

            print(f"[arena] presize: budget {budget / 1e9:.1f} GB, {len(fits)} fits, batch rows {rows:.3g} T {T} -> "
                  f"slot {need / 1e9:.1f} GB", file=sys.stderr, flush=True)
        forest_ops.ARENA.reserve(data.device, "forest", need)

    def _budget(self, data) -> float:
        if self.hbm_budget_bytes:
            return float(self.hbm_budget_bytes)
        env = os.environ.get("DML_HBM_BUDGET_GB")   # Config.hbm_budget_gb
        if env:
            return float(env) * 1e9
        if data.is_gpu:
            free, _total = torch.cuda.mem_get_info(data.device)
            # blocks the caching allocator holds but nobody uses are free for this batch too
            # (without this, the previous batch's freed pool makes the next batch split)
            cached = torch.cuda.memory_reserved(data.device) - torch.cuda.memory_allocated(data.device)
            # ... and so are the idle forest arena slots this batch will reuse (ops/forest_ops.py)
            arena = forest_ops.ARENA.held_bytes(data.device)
            return float(os.environ.get("DML_HBM_FRACTION", "0.55")) * (free + max(0, cached) + arena)
        return 8e9

    def run(self, data, tasks: List[FitTask], keep_models: bool = False) -> List[FitOutput]:
        if not tasks:
            return []
        is_reg = not data.classification
        if is_reg and any(t.params.get("criterion") == forest_ops.POISSON for t in tasks):
            ymin = float(data.y_reg.min()) if data.n else 0.0
            if getattr(data, "is_row_shard", False):
                ymin = float(data.all_reduce(torch.tensor([ymin], dtype=torch.float64, device=data.device), "min")[0])
            if ymin < 0:   # sklearn raises the same
                raise ParamError("Some value(s) of y are negative which is not allowed for Poisson regression.")
        with trace.range("forest_plan"):
            Xb = data.binned()
        sharded = getattr(data, "is_row_shard", False)
        if sharded:
            # the row-sharded builder sums histograms (medians need every row) and keeps no node
            # bounds: the cluster runner sends such jobs task-parallel (parallel/runner.py
            # needs_whole_rows); never grow a different estimator than the one requested
            for t in tasks:
                if t.params.get("criterion") == forest_ops.MAE or t.params.get("monotonic_cst") is not None:
                    raise ParamError("criterion='absolute_error' and monotonic_cst need every row on one rank: "
                                     "run this job with parallelism='task'")
        # absolute_error trees grow on their own builder (forest_mae.hip / forest_cpu.cpp): batch them apart
        tasks_in = tasks
        # fits differing only in n_estimators with an explicit random_state grow the same first
        # trees: only the largest is grown, the others predict from its first trees (base.py)
        follow: Dict[int, List[FitTask]] = {}
        if not sharded:   # on the GPU predictor also max_depth prefixes (depth-capped predicts)
            tasks, follow = prefix_groups(tasks, depth=data.is_gpu)
        tasks = sorted(tasks, key=_host_only)
        with trace.range("forest_budget"):
            budget = self._budget(data)
        if sharded:   # every rank must form the SAME batches: the smallest budget of the group
            budget = float(data.all_reduce(torch.tensor([budget], dtype=torch.float64, device=data.device), "min")[0])
        # row shard: trees per level-synchronous build -- the (tree, row) pair arrays take
        # ~26 B per tree and local row (ops/forest_dp.py build_dp tree_chunk)
        tree_chunk = max(1, int(budget // max(1.0, data.n * 26.0))) if sharded else None
        outs: Dict[int, FitOutput] = {}
        # batches of whole fits under the memory budget (on the device: the builder's real
        # workspace + node-pool bytes, the same rule ``presize`` sizes the arena with)
        batches: List[List[FitTask]] = []
        cur, cur_bytes = [], 0.0
        rows = pool = 0.0
        T = 0
        for t in tasks:
            if cur and _host_only(t) != _host_only(cur[-1]):
                batches.append(cur)
                cur, cur_bytes, rows, T, pool = [], 0.0, 0.0, 0, 0.0
            if sharded:
                b = self._dp_bytes(data, t.params)
                if cur and cur_bytes + b > budget:
                    batches.append(cur)
                    cur, cur_bytes = [], 0.0
                cur.append(t)
                cur_bytes += b
                continue
            if data.is_gpu:
                fr, fp = self.footprint(data, t.params)
                ft = t.params["n_estimators"]
                if cur and self._need(data, rows + fr, T + ft, pool + fp) > budget:
                    batches.append(cur)
                    cur, rows, T, pool = [], 0.0, 0, 0.0
                cur.append(t)
                rows, T, pool = rows + fr, T + ft, pool + fp
                continue
            b = self._tree_bytes(data, t.params) * t.params["n_estimators"]
            if cur and cur_bytes + b > budget:
                batches.append(cur)
                cur, cur_bytes = [], 0.0
            cur.append(t)
            cur_bytes += b
        if cur:
            batches.append(cur)
        if os.environ.get("DML_ARENA_LOG") and data.is_gpu:
            import sys

            print(f"[arena] run: budget {budget / 1e9:.1f} GB, {len(tasks)} fits -> {len(batches)} batches "
                  f"{[len(b) for b in batches]}", file=sys.stderr, flush=True)
        for batch in batches:
            with trace.range("forest_batch"):
                out_b = self._run_batch(data, Xb, batch, is_reg, keep_models, tree_chunk, follow)
            for o in out_b:
                outs[o.task_id] = o
        return [outs[t.task_id] for t in tasks_in]

    def _dp_bytes(self, data, rp) -> float:
        """Device bytes of one fit under the row-sharded builder: the (tree, row) weight
        table and the sorted pair arrays of the local rows (3 int32 + sort scratch), and
        the fit's share of the replicated node pool (ops/forest_dp.py)."""
        T = rp["n_estimators"]
        _rows, pool = self.footprint(data, rp)
        VC = data.n_classes if data.classification else 3
        return T * data.n * (1 + 0.632 * 40) + pool * (8 + 8 * VC) * 2

    def _specs(self, batch: List[FitTask]) -> np.ndarray:
        T = sum(t.params["n_estimators"] for t in batch)
        specs = forest_ops.make_specs(T)
        i = 0
        for f, t in enumerate(batch):
            rp = t.params
            base = rp["seed"] if rp["seed"] is not None else t.seed
            n = rp["n_estimators"]
            sl = specs[i:i + n]
            sl["seed"] = [native_seed(base, j) for j in range(n)]
            sl["split"] = t.split
            sl["fit"] = f
            sl["max_depth"] = rp["max_depth"]
            sl["min_samples_split"] = rp["min_samples_split"]
            sl["min_samples_leaf"] = rp["min_samples_leaf"]
            sl["max_features"] = rp["max_features"]
            sl["bootstrap"] = rp["bootstrap"]
            sl["criterion"] = rp["criterion"]
            sl["min_impurity_decrease"] = rp["min_impurity_decrease"]
            sl["min_weight_frac"] = rp.get("min_weight_fraction_leaf", 0.0)
            sl["pois_cdf"] = native.poisson_cdf_table(rp["lambda"])
            cw = rp.get("class_weight")
            sl["cw_mode"] = 0 if cw is None else (2 if cw == "balanced_subsample" else 1)
            i += n
        return specs

    @staticmethod
    def class_weight_table(data, batch: List[FitTask], specs: np.ndarray):
        """[T, C] class weights per tree (sklearn semantics) or None when no fit uses them.
        ``balanced``: n_train / (n_classes_present * n_k) over the fit's training rows;
        a dict maps class labels to weights (missing classes 1); ``balanced_subsample``
        rows are computed per tree on the device from its bootstrap counts."""
        if not any(t.params.get("class_weight") is not None for t in batch) or not data.classification:
            return None
        C = data.n_classes
        tab = np.ones((len(specs), C), dtype=np.float64)
        labels = [str(c) for c in np.asarray(data.classes).tolist()]
        i = 0
        for t in batch:
            n = t.params["n_estimators"]
            cw = t.params.get("class_weight")
            row = np.ones(C, dtype=np.float64)
            if cw == "balanced":   # global counts under a row shard (an all-reduce)
                cnt = data.train_class_counts(t.split, C).cpu().numpy().astype(np.float64)
                present = max(1, int((cnt > 0).sum()))
                row = np.where(cnt > 0, float(cnt.sum()) / (present * np.maximum(cnt, 1)), 1.0)
            elif isinstance(cw, dict):
                for k, lab in enumerate(labels):
                    if lab in cw:
                        row[k] = float(cw[lab])
                    elif lab.lstrip("-").isdigit() and str(int(lab)) in cw:
                        row[k] = float(cw[str(int(lab))])
            tab[i:i + n] = row
            i += n
        return tab

    def _early_predict(self, data, Xb, batch: List[FitTask], is_reg: bool, mono):
        """(make, done) for build_gpu's early predict, or None: fit f of depth-limited trees
        is complete after builder level max_depth - 1."""
        if os.environ.get("DML_EARLY_PREDICT", "1") == "0" or not _early_ok(data, batch, is_reg, mono):
            return None
        done = np.array([t.params["max_depth"] - 1 if t.params["max_depth"] < forest_ops.INT32_MAX else 1 << 30
                         for t in batch], dtype=np.int32)
        if not np.any(done < (1 << 30)):
            return None
        toff = np.zeros(len(batch) + 1, dtype=np.int64)
        np.cumsum([t.params["n_estimators"] for t in batch], out=toff[1:])
        rows = [data.test_rows[t.split] for t in batch]
        roff = np.zeros(len(batch) + 1, dtype=np.int64)
        np.cumsum([int(r.numel()) for r in rows], out=roff[1:])
        rows_cat = torch.cat(rows) if rows else torch.empty(0, dtype=torch.int32, device=data.device)
        want_proba = (not is_reg) and any(t.need_proba for t in batch)
        C = data.n_classes
        VC = 3 if is_reg else C
        def make(nodes, vals):
            return forest_ops.GpuPredict(nodes, vals, VC, is_reg, C, Xb, toff, roff, rows_cat, want_proba)

        return make, done

    def _run_batch(self, data, Xb, batch: List[FitTask], is_reg: bool, keep_models: bool,
                   tree_chunk: int | None = None, follow: Optional[Dict[int, List[FitTask]]] = None
                   ) -> List[FitOutput]:
        specs = self._specs(batch)
        cw = self.class_weight_table(data, batch, specs)
        t0 = time.perf_counter()
        sharded = getattr(data, "is_row_shard", False)
        if sharded:
            from ..ops import forest_dp

            fb = forest_dp.build_dp(Xb, data.y_cls, None if not is_reg else data.y_reg, data.roles, specs,
                                    data.n_classes, is_reg, data.r0, reduce=data.all_reduce, cw=cw, comm=data,
                                    tree_chunk=tree_chunk)
        elif _host_only(batch[0]) and data.is_gpu and os.environ.get("DML_MAE_GPU", "1") != "0":
            # absolute_error on the GPU: the MAE builder (forest_mae.hip), node for node the
            # host builder's trees (rows in target order, exact fixed-point abs deviations)
            fb = forest_ops.build_gpu_mae(Xb, data.y_reg, data.roles, specs)
        elif _host_only(batch[0]):
            # exact absolute_error (per-node weighted medians) on the host builder (CPU data,
            # or DML_MAE_GPU=0); the pruning / refine / predict steps below run where the data lives
            mono = _mono_table(batch, Xb.shape[1], is_reg)
            ycls = None if is_reg else np.asarray(data.y_enc, dtype=np.int32)
            fb = forest_ops.build_cpu(Xb.cpu().numpy(), ycls, None if not is_reg else data.y_reg.cpu().numpy(),
                                      data.roles_np(), specs, data.n_classes, is_reg, cw=cw, mono=mono)
            if data.is_gpu:
                fb.nodes = torch.from_numpy(fb.nodes).to(data.device)
                fb.vals = torch.from_numpy(fb.vals).to(data.device)
        elif data.is_gpu:
            # monotonic_cst grows on the HIP builder too (per-node bounds in every tier)
            mono = _mono_table(batch, Xb.shape[1], is_reg)
            early = self._early_predict(data, Xb, batch, is_reg, mono)
            fb = forest_ops.build_gpu(Xb, data.y_cls, None if not is_reg else data.y_reg, data.roles, specs,
                                      data.n_classes, is_reg, self.tiers, reuse_pool=True,
                                      XbT=data.binned_feature_major(), cw=cw, mono=mono, early_predict=early)
        else:
            fb = forest_ops.build_cpu(Xb.numpy(), data.y_enc, None if not is_reg else data.y_reg.numpy(),
                                      data.roles_np(), specs, data.n_classes, is_reg, cw=cw,
                                      mono=_mono_table(batch, Xb.shape[1], is_reg))
        try:
            if any(t.params.get("max_leaf_nodes") for t in batch):
                with trace.range("forest_prune"):
                    forest_ops.prune_max_leaves(fb, specs, np.repeat(
                        [t.params.get("max_leaf_nodes", 0) for t in batch], [t.params["n_estimators"] for t in batch]))
            if any(t.params.get("ccp_alpha", 0.0) > 0 for t in batch):
                with trace.range("forest_ccp"):   # sklearn prunes after growing (and after best-first)
                    forest_ops.prune_ccp(fb, specs, np.repeat(
                        [t.params.get("ccp_alpha", 0.0) for t in batch], [t.params["n_estimators"] for t in batch]))
            with trace.range("forest_refine"):
                if sharded:
                    from ..ops import forest_dp

                    vals, exact = data.bin_values()
                    if bool(exact.any()):   # already the AND over ranks: the same answer on every rank
                        forest_dp.refine_dp(fb, Xb, data.roles, specs, data.r0, vals, exact, reduce=data.all_reduce)
                else:
                    _refine(data, fb, Xb, specs, data.roles)
            toff = np.zeros(len(batch) + 1, dtype=np.int64)
            np.cumsum([t.params["n_estimators"] for t in batch], out=toff[1:])
            rows = [data.test_rows[t.split] for t in batch]
            roff = np.zeros(len(batch) + 1, dtype=np.int64)
            np.cumsum([int(r.numel()) for r in rows], out=roff[1:])
            want_proba = (not is_reg) and any(t.need_proba for t in batch)
            proba = None
            gp = getattr(fb, "predict", None)
            if gp is not None:
                # the builder already predicted the fits whose trees were complete before the
                # last level (ForestArgs.early_pred); the deeper ones are predicted here
                done = fb.early_done
                gp.run([f for f in range(len(batch)) if done[f] != -2])
                pred = gp.result()
            elif data.is_gpu:
                rows_cat = torch.cat(rows) if rows else torch.empty(0, dtype=torch.int32, device=data.device)
                pred = forest_ops.predict(fb, Xb, toff, roff, rows_cat, want_proba=want_proba)
            else:
                rows_cat = np.concatenate([r.numpy() for r in rows]) if rows else np.zeros(0, np.int32)
                pred = forest_ops.predict(fb, Xb.numpy(), toff, roff, rows_cat, want_proba=want_proba)
                pred = (torch.from_numpy(pred[0]), torch.from_numpy(pred[1])) if want_proba else torch.from_numpy(pred)
            if want_proba:   # sklearn predict_proba: the mean of the trees' leaf class fractions
                pred, proba = pred
            if data.is_gpu:
                with trace.range("forest_predict_wait"):   # refine + predict kernels drain here
                    torch.cuda.synchronize(data.device)
            dt = time.perf_counter() - t0
            total_trees = max(1, int(toff[-1]))
            outs = []
            for f, t in enumerate(batch):
                share = t.params["n_estimators"] / total_trees
                o = FitOutput(task_id=t.task_id, pred=pred[roff[f]:roff[f + 1]], fit_seconds=dt * share,
                              proba=None if proba is None else proba[roff[f]:roff[f + 1]],
                              info={"warnings": t.params.get("warnings", []), "batch_stats": dict(fb.stats)})
                if keep_models and t.keep:
                    o.model = extract_forest(fb, int(toff[f]), int(toff[f + 1]), data, t)
                outs.append(o)
                for fo in (follow or {}).get(t.task_id, []):   # prefix fits: leader f's first m trees
                    m = int(fo.params["n_estimators"])
                    # ... read down to the follower's max_depth when it is shallower (0: whole trees)
                    cap = int(fo.params["max_depth"]) if fo.params["max_depth"] < t.params["max_depth"] else 0
                    toff_f = np.array([toff[f], toff[f] + m], dtype=np.int64)
                    roff_f = np.array([0, int(rows[f].numel())], dtype=np.int64)
                    if data.is_gpu:
                        pf = forest_ops.predict(fb, Xb, toff_f, roff_f, rows[f], want_proba=want_proba,
                                                depth_cap=np.array([cap], dtype=np.int32) if cap else None)
                    else:
                        pf = forest_ops.predict(fb, Xb.numpy(), toff_f, roff_f, rows[f].numpy(), want_proba=want_proba)
                        pf = ((torch.from_numpy(pf[0]), torch.from_numpy(pf[1])) if want_proba
                              else torch.from_numpy(pf))
                    pf, prf = pf if want_proba else (pf, None)
                    of = FitOutput(task_id=fo.task_id, pred=pf, proba=prf, fit_seconds=dt * m / total_trees,
                                   info={"warnings": fo.params.get("warnings", []), "batch_stats": dict(fb.stats),
                                         "prefix_of": t.task_id})
                    if keep_models and fo.keep:
                        of.model = extract_forest(fb, int(toff[f]), int(toff[f]) + m, data, fo, depth_cap=cap)
                    outs.append(of)
            return outs
        finally:   # the node pool is an arena slot: free it for the next batch
            forest_ops.release_pool(fb)


def _early_ok(data, batch: List[FitTask], is_reg: bool, mono) -> bool:
    """A batch whose fits can be predicted by the builder as soon as their trees are
    complete: nothing rewrites the trees after growth (no max_leaf_nodes / ccp pruning, no
    monotonic clip, no midpoint refinement of exactly-binned features)."""
    if mono is not None or any(t.params.get("max_leaf_nodes") or t.params.get("ccp_alpha", 0.0) > 0 for t in batch):
        return False
    if getattr(data, "_refine_needed", None) is None:
        _vals, exact = data.bin_values()
        data._refine_needed = bool(exact.any())
    return not data._refine_needed


def _host_only(t: FitTask) -> bool:
    """absolute_error trees grow on the host builder (per-node weighted medians)."""
    return t.params.get("criterion") == forest_ops.MAE


def _mono_table(batch, d: int, is_reg: bool):
    """int8 [fits][d] monotonic_cst rows of a batch (None: no fit is constrained);
    classifier rows constrain the class-0 fraction, so they are negated."""
    if not any(t.params.get("monotonic_cst") is not None for t in batch):
        return None
    mono = np.zeros((len(batch), d), dtype=np.int8)
    for f, t in enumerate(batch):
        if t.params.get("monotonic_cst") is not None:
            mono[f] = np.asarray(t.params["monotonic_cst"], dtype=np.int8) * (1 if is_reg else -1)
    return mono


def _refine(data, fb, Xb, specs, roles) -> None:
    """sklearn midpoint thresholds where the binning is exact (no-op on quantile-binned data)."""
    vals, exact = data.bin_values()
    # cached per dataset: a device-side any() per call is a host/GPU sync (boosting calls
    # this once per stage)
    if getattr(data, "_refine_needed", None) is None:
        data._refine_needed = bool(exact.any())
    if not data._refine_needed:
        return
    if data.is_gpu:
        forest_ops.refine_thresholds(fb, Xb, specs, roles, vals, exact)
    else:
        forest_ops.refine_thresholds(fb, Xb.numpy(), specs, roles.numpy() if isinstance(roles, torch.Tensor) else roles,
                                     vals.numpy(), exact.numpy())


def native_seed(base: int, tree: int) -> int:
    x = (int(base) * 0x9E3779B97F4A7C15 + tree * 0xBF58476D1CE4E5B9 + 0x1234567) & 0xFFFFFFFFFFFFFFFF
    x ^= x >> 31
    return x


def extract_forest(fb, t0: int, t1: int, data, task: FitTask, depth_cap: int = 0) -> Dict[str, Any]:
    """Renumber trees [t0, t1) of a batch pool into a standalone forest in pool layout.

    Layout matches the kernels' contract: tree j's root is node j, every other node
    follows, children pairs adjacent -- so the saved model predicts with the same
    HIP/C++ predictors (``roots`` is kept for readability).  The renumbering is
    breadth-first and vectorised level by level on the pool's own device (a full-depth
    forest on 1M rows has ~10^8 nodes: a per-node host loop would take minutes), and only
    the extracted nodes leave the device.  ``depth_cap`` > 0 keeps the top depth_cap levels
    (nodes at that depth become leaves with their stored sums: a max_depth prefix fit).
    """
    nodes = fb.nodes if isinstance(fb.nodes, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(fb.nodes))
    vals = fb.vals if isinstance(fb.vals, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(fb.vals))
    dev = nodes.device
    T = t1 - t0
    order, lefts, splits = [], [], []
    fo = torch.arange(t0, t1, dtype=torch.int64, device=dev)
    nxt = T
    level = 0
    while fo.numel():
        rec = nodes[fo]
        internal = rec[:, 0] >= 0
        if depth_cap > 0 and level >= depth_cap:
            internal = torch.zeros_like(internal)
        k = int(internal.sum())
        left_new = torch.full((fo.numel(),), -1, dtype=torch.int32, device=dev)
        left_new[internal] = (nxt + 2 * torch.arange(k, device=dev)).to(torch.int32)
        order.append(fo)
        lefts.append(left_new)
        splits.append(torch.where(internal, rec[:, 0], torch.full_like(rec[:, 0], -1)))
        level += 1
        l_old = rec[internal, 1].to(torch.int64)
        fo = torch.stack([l_old, l_old + 1], 1).reshape(-1)   # children pairs stay adjacent
        nxt += 2 * k
    old = torch.cat(order)
    nn = torch.stack([torch.cat(splits), torch.cat(lefts)], 1).cpu().numpy().astype(np.int32)
    vv = vals[old].cpu().numpy().astype(np.float64)
    return {
        "kind": "forest",
        "is_reg": bool(fb.is_reg),
        "n_classes": int(fb.n_classes),
        "classes": None if data.classes is None else np.asarray(data.classes).tolist(),
        "nodes": nn,
        "vals": vv,
        "n_trees": T,
        "edges": data.edges.cpu().numpy(),
        "n_features": int(data.d),
        "params": {k: v for k, v in task.params.items() if k != "warnings"},
        "model_type": task.model_type,
    }


register(ForestFamily())
