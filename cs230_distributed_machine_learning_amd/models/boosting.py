"""GradientBoosting{Classifier,Regressor} — every fit of a job boosted in lock-step.

Reference: both are whitelisted estimators (aws-prod/worker/worker.py:41,48) that
sklearn fits one (candidate, fold) at a time: ``n_estimators`` sequential stages, each
fitting ``K`` depth-``max_depth`` regression trees to the negative gradient and then
re-solving the leaf values with one Newton / quantile step (sklearn
``ensemble/_gb.py`` ``_fit_stage`` / ``_update_terminal_regions``).

Here stage ``s`` of EVERY fit in the batch (candidates x CV folds x holdout x K
classes) is one call of the batched histogram tree builder (csrc/kernels/forest.hip,
regression mode) on a ``[fits*K, n]`` pseudo-residual matrix (``ForestArgs.ystride``:
each tree reads its own target row), followed by one ``dml_forest_apply`` launch that
maps every row to its leaf in every new tree.  Leaf line searches are segmented
reductions over (tree, leaf) and the raw scores of all rows (train and held-out) are
updated in place, so held-out predictions are ready when the last stage ends.

Semantics kept from sklearn: losses log_loss (binomial / multinomial with the
(K-1)/K factor), exponential, squared_error, absolute_error, huber, quantile; the
DummyEstimator initial predictions; ``friedman_mse`` (same split ranking as
squared_error for unit weights); learning_rate, subsample (exactly
``int(subsample * n_train)`` in-bag rows per stage, drawn on-device), max_depth,
min_samples_split/leaf, min_impurity_decrease, max_features.  Split thresholds come
from the 256-bin quantisation shared with the forests (exact whenever a feature has
<= 256 distinct values); early stopping (``n_iter_no_change``) holds out sklearn's
validation split and stops on sklearn's rule
and is reported in the subtask's warnings.
"""
from __future__ import annotations

import ctypes
import math
import os
import threading
import time
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from ..ops import forest_ops
from ..search import cv as cv_mod
from ..utils import native
from .base import (Family, FitOutput, FitTask, ParamError, as_bool, as_float, as_int, prefix_groups, register,
                   seed_of)
from .forest import _count_param, _refine, native_seed

_CLS = "GradientBoostingClassifier"
_REG = "GradientBoostingRegressor"

LOSS_SQ, LOSS_ABS, LOSS_HUBER, LOSS_QUANT, LOSS_LOG, LOSS_EXP = range(6)
_CLS_LOSSES = {"log_loss": LOSS_LOG, "deviance": LOSS_LOG, "exponential": LOSS_EXP}
_REG_LOSSES = {"squared_error": LOSS_SQ, "ls": LOSS_SQ, "absolute_error": LOSS_ABS, "lad": LOSS_ABS,
               "huber": LOSS_HUBER, "quantile": LOSS_QUANT}

_DEFAULTS = {
    "loss": None, "learning_rate": 0.1, "n_estimators": 100, "subsample": 1.0, "criterion": "friedman_mse",
    "min_samples_split": 2, "min_samples_leaf": 1, "min_weight_fraction_leaf": 0.0, "max_depth": 3,
    "min_impurity_decrease": 0.0, "init": None, "random_state": None, "max_features": None, "alpha": 0.9,
    "verbose": 0, "max_leaf_nodes": None, "warm_start": False, "validation_fraction": 0.1,
    "n_iter_no_change": None, "tol": 1e-4, "ccp_alpha": 0.0,
}
_F32_EPS = float(np.finfo(np.float32).eps)


def _max_features(v, d):
    if v is None or v == "None":
        return d
    if isinstance(v, str):
        if v in ("sqrt", "auto"):
            return max(1, int(math.sqrt(d)))
        if v == "log2":
            return max(1, int(math.log2(d)))
        raise ParamError(f"max_features {v!r} not understood")
    if isinstance(v, bool):
        raise ParamError("max_features must not be a bool")
    if isinstance(v, int):
        return max(1, min(d, v))
    f = float(v)
    if not 0.0 < f <= 1.0:
        raise ParamError(f"max_features fraction must be in (0, 1], got {f}")
    return max(1, int(f * d))


# ---- percentiles (numpy 'linear' for the initial estimate, sklearn inverted-CDF in leaves) ----
_LANE_STREAMS: Dict[Any, List[Any]] = {}   # device -> the boosting lanes' streams (made once)


def sharded_pct_ok() -> bool:
    """The row-sharded fused stage (phased gbrt.hip entry points) is in the loaded library."""
    try:
        lib = native.hip_lib()
    except Exception:
        return False
    return all(getattr(lib, f, None) is not None for f in ("dml_gb_stage_phase", "dml_gb_sel_step",
                                                           "dml_gb_fit_sel_step"))


def _radix_select(step, args, stream, data, hist: torch.Tensor, finish: int = -1) -> None:
    """The exact 8-pass radix select of gbrt.hip over every rank's rows: each pass counts this
    rank's keys' next byte, the counters are summed over the ranks, and every rank picks the
    same byte from the sums (so all ranks hold the same percentile)."""
    def call(which, shift):
        rc = step(ctypes.byref(args), which, shift, stream)
        if rc:
            raise RuntimeError(f"gbrt select step {which} failed ({rc})")

    call(0, 56)
    for shift in range(56, -1, -8):
        call(1, shift)
        data.all_reduce(hist)
        call(2, shift)
    if finish >= 0:
        call(finish, 0)


def _sharded_stage(lib, sa, stream, data, slot_sum: torch.Tensor, sel_hist: Optional[torch.Tensor], newton: bool,
                   huber: bool) -> None:
    """Leaf line search + raw update of a row-sharded stage: the fused kernels in phases, with
    the per-leaf Newton / huber sums and the percentile select's byte counts all-reduced."""
    def phase(p):
        sa.phase = p
        rc = lib.dml_gb_stage_phase(ctypes.byref(sa), stream)
        if rc:
            raise RuntimeError(f"dml_gb_stage_phase({p}) failed ({rc})")

    phase(1)                                         # leaf slots, local Newton sums
    if sel_hist is not None:                         # leaf percentiles over every rank's rows
        _radix_select(lib.dml_gb_sel_step, sa, stream, data, sel_hist)
        if huber:
            phase(3)                                 # local clipped-deviation sums
    if newton or huber:
        data.all_reduce(slot_sum)
    phase(2)                                         # leaf values + raw update of the local rows
    sa.phase = 0


def _percentile_linear(v: torch.Tensor, q: float) -> torch.Tensor:
    s, _ = torch.sort(v)
    m = s.numel()
    pos = q * (m - 1)
    lo = int(math.floor(pos))
    hi = min(lo + 1, m - 1)
    return s[lo] + (s[hi] - s[lo]) * (pos - lo)


def _percentile_icdf(v: torch.Tensor, q: float) -> torch.Tensor:
    """sklearn ``_weighted_percentile`` with unit weights (lower value on ties)."""
    s, _ = torch.sort(v)
    m = s.numel()
    i = max(0, min(m - 1, int(math.ceil(q * m - 1e-12)) - 1))
    return s[i]


def _segment_percentile(seg: torch.Tensor, val: torch.Tensor, n_seg: int, q: float) -> torch.Tensor:
    """Inverted-CDF percentile of ``val`` within each segment id (unit weights); NaN if empty."""
    out = torch.full((n_seg,), float("nan"), dtype=val.dtype, device=val.device)
    if seg.numel() == 0:
        return out
    order = torch.argsort(val, stable=True)
    seg_s = seg[order]
    order2 = torch.argsort(seg_s, stable=True)
    seg_sorted = seg_s[order2]
    val_sorted = val[order][order2]
    cnt = torch.bincount(seg_sorted, minlength=n_seg)
    start = torch.cumsum(cnt, 0) - cnt
    has = cnt > 0
    k = torch.clamp(torch.ceil(q * cnt.double() - 1e-12).long() - 1, min=0)
    k = torch.minimum(k, (cnt - 1).clamp_min(0))
    idx = (start + k)[has]
    out[has] = val_sorted[idx]
    return out


class GradientBoostingFamily(Family):
    model_types = (_CLS, _REG)
    classifiers = (_CLS,)

    binned_ok = True   # the stages only read the uint8 bins (DeviceData binned_only tables)
    data_parallel = True   # row-sharded stages: ops/forest_dp.py trees + all-reduced line searches
    dp_when_few = False

    def __init__(self):
        self.tiers = forest_ops.ForestTiers()

    def resolve(self, model_type, params, n_train, n_features, n_classes) -> Dict[str, Any]:
        p = dict(_DEFAULTS)
        p.update({k: v for k, v in params.items() if k in _DEFAULTS})
        is_cls = model_type == _CLS
        warn: List[str] = []
        unknown = sorted(k for k in params if k not in _DEFAULTS)
        if unknown:
            warn.append(f"ignored unknown parameters {unknown}")
        loss_name = p["loss"] or ("log_loss" if is_cls else "squared_error")
        table = _CLS_LOSSES if is_cls else _REG_LOSSES
        if loss_name not in table:
            raise ParamError(f"loss {loss_name!r} invalid for {model_type}")
        loss = table[loss_name]
        if loss == LOSS_EXP and n_classes > 2:
            raise ParamError(f"ExponentialLoss requires 2 classes; got {n_classes} class(es).")
        if p["criterion"] not in ("friedman_mse", "squared_error"):
            raise ParamError(f"criterion {p['criterion']!r} invalid")
        lr = as_float(p["learning_rate"], "learning_rate", lo=0.0)
        sub = as_float(p["subsample"], "subsample", lo=0.0, hi=1.0)
        if sub <= 0:
            raise ParamError("subsample must be in (0, 1]")
        init = p["init"]
        if init not in (None, "zero", "None"):
            raise ParamError("init must be None or 'zero' (custom init estimators are not supported)")
        nic = as_int(p["n_iter_no_change"], "n_iter_no_change", lo=1, allow_none=True)
        vf = as_float(p["validation_fraction"], "validation_fraction", lo=0.0, hi=1.0)
        if nic is not None and not 0.0 < vf < 1.0:
            raise ParamError("validation_fraction must be in (0, 1)")
        rs = p["random_state"]
        rs = int(rs) if isinstance(rs, (int, np.integer)) or (isinstance(rs, str) and rs.lstrip("-").isdigit()) else None
        ccp = as_float(p["ccp_alpha"], "ccp_alpha", lo=0.0)
        mwf = as_float(p["min_weight_fraction_leaf"], "min_weight_fraction_leaf", lo=0.0, hi=0.5)
        alpha = as_float(p["alpha"], "alpha", lo=0.0, hi=1.0)
        if loss in (LOSS_HUBER, LOSS_QUANT) and not 0.0 < alpha < 1.0:
            raise ParamError("alpha must be in (0, 1)")
        md = as_int(p["max_depth"], "max_depth", lo=1, allow_none=True)
        return {
            "loss": loss, "learning_rate": lr, "n_estimators": as_int(p["n_estimators"], "n_estimators", lo=1,
                                                                      hi=100000),
            "subsample": sub, "max_depth": md if md is not None else forest_ops.INT32_MAX,
            "min_samples_split": _count_param(p["min_samples_split"], n_train, "min_samples_split", 2),
            "min_samples_leaf": _count_param(p["min_samples_leaf"], n_train, "min_samples_leaf", 1),
            "min_impurity_decrease": as_float(p["min_impurity_decrease"], "min_impurity_decrease", lo=0.0),
            "max_features": _max_features(p["max_features"], n_features), "alpha": alpha,
            "init_zero": init == "zero", "seed": seed_of(p["random_state"]), "warnings": warn,
            "ccp_alpha": ccp, "min_weight_fraction_leaf": mwf,
            "criterion": forest_ops.FRIEDMAN if p["criterion"] == "friedman_mse" else forest_ops.MSE,
            "n_iter_no_change": nic, "validation_fraction": vf, "tol": as_float(p["tol"], "tol", lo=0.0),
            "random_state_int": rs,
            "max_leaf_nodes": as_int(p["max_leaf_nodes"] if p["max_leaf_nodes"] != "None" else None, "max_leaf_nodes",
                                     lo=2, allow_none=True) or 0,
        }

    def cost(self, model_type, rp, n_train, n_features, n_classes) -> float:
        K = n_classes if n_classes > 2 else 1
        depth = min(rp["max_depth"], 12)
        return rp["n_estimators"] * K * n_train * rp["subsample"] * depth * rp["max_features"] * 2e-9 + 1e-2

    def run(self, data, tasks: List[FitTask], keep_models: bool = False) -> List[FitOutput]:
        if not tasks:
            return []
        K = data.n_classes if (data.classification and data.n_classes > 2) else 1
        per_fit = K * data.n * (8 + 4 + 4 + 1) * 1.5
        budget = 0.4 * torch.cuda.mem_get_info(data.device)[0] if data.is_gpu else 4e9
        if getattr(data, "is_row_shard", False):   # every rank must cut the same batches
            budget = float(data.all_reduce(torch.tensor([budget], dtype=torch.float64, device=data.device), "min")[0])
        cap = max(1, int(budget // max(1.0, per_fit)))
        # fits differing only in n_estimators (explicit random_state, no early stopping): the
        # longest one is boosted, the shorter ones are its stage prefixes (models/base.py)
        leaders, follow = prefix_groups(tasks, ok=lambda t: not t.params.get("n_iter_no_change"))
        outs: Dict[int, FitOutput] = {}
        for i in range(0, len(leaders), cap):
            for o in self._boost_lanes(data, leaders[i:i + cap], K, keep_models, follow):
                outs[o.task_id] = o
        return [outs[t.task_id] for t in tasks]

    def _boost_lanes(self, data, batch: List[FitTask], K: int, keep_models: bool,
                     follow: Optional[Dict[int, List[FitTask]]] = None) -> List[FitOutput]:
        """A device batch split over build LANES (DML_GB_LANES, default 3): each lane boosts its
        share of the fits from its own host thread on its own stream.  A stage is a chain of
        short launches with a host read-back per tree level; with one lane the GPU idles during
        every read-back, with two the other lane's kernels run meanwhile.  Fits are independent,
        so the results are those of one lane (same kernels, same order inside each fit)."""
        lanes = max(1, min(4, int(os.environ.get("DML_GB_LANES", "3"))))
        if (not data.is_gpu or getattr(data, "is_row_shard", False) or lanes < 2 or len(batch) < 2
                or getattr(native.hip_lib(), "dml_forest_set_lane", None) is None):
            return self._boost(data, batch, K, keep_models, follow)
        lanes = min(lanes, len(batch))
        # each lane holds its own workspace arena slot and whole-histogram buffers for its share
        # of the batch (the batch cap in ``run`` prices one build): drop lanes until the batch
        # state plus every lane's workspace fits the free HBM
        per_fit = K * data.n * (8 + 4 + 4 + 1) * 1.5
        free = torch.cuda.mem_get_info(data.device)[0]
        lane_ws = lambda L: 2.0 * per_fit * (-(-len(batch) // L)) + (256 << 20)   # noqa: E731
        while lanes > 1 and len(batch) * per_fit + lanes * lane_ws(lanes) > 0.9 * free:
            lanes -= 1
        if lanes < 2:
            return self._boost(data, batch, K, keep_models, follow)
        # longest-processing-time split of the fits (stage count x depth x trees per stage)
        w = [t.params["n_estimators"] * max(1, min(t.params["max_depth"], 12)) for t in batch]
        groups: List[List[int]] = [[] for _ in range(lanes)]
        load = [0] * lanes
        for i in sorted(range(len(batch)), key=lambda i: -w[i]):
            g = load.index(min(load))
            groups[g].append(i)
            load[g] += w[i]
        groups = [sorted(g) for g in groups if g]
        # lazily built per-dataset state, made once here (not raced by the lanes)
        data.binned()
        if hasattr(data, "binned_feature_major"):
            data.binned_feature_major()
        data.bin_values()
        dev = data.device
        main = torch.cuda.current_stream(dev)
        # the lanes' streams are made once per device and reused by every later batch: streams
        # drawn fresh from torch's pool land on other hardware queues each time, and a job whose two
        # lane streams shared a queue with each other (or with the builder's side streams) ran ~40 %
        # slower (the second of back-to-back config-6 jobs: 1.53 vs 1.08 s,
        # profiles/r5_gbrt_cfg6_back_to_back.txt)
        pool = _LANE_STREAMS.setdefault(dev, [])
        while len(pool) < len(groups):
            pool.append(torch.cuda.Stream(dev))
        streams = pool[:len(groups)]
        results: List[Any] = [None] * len(groups)
        errors: List[Any] = [None] * len(groups)

        def work(li: int) -> None:
            try:
                forest_ops.set_build_lane(li)
                streams[li].wait_stream(main)
                with torch.cuda.device(dev), torch.cuda.stream(streams[li]):
                    results[li] = self._boost(data, [batch[i] for i in groups[li]], K, keep_models, follow)
            except BaseException as e:   # re-raised on the caller's thread
                errors[li] = e
            finally:
                forest_ops.set_build_lane(0)

        threads = [threading.Thread(target=work, args=(li,), name=f"gb-lane{li}", daemon=True)
                   for li in range(1, len(groups))]
        for th in threads:
            th.start()
        work(0)
        for th in threads:
            th.join()
        for st in streams:
            main.wait_stream(st)
        for e in errors:
            if e is not None:
                raise e
        return [o for res in results for o in res]   # leaders and their prefix fits (run orders them)

    # ------------------------------------------------------------------------------------
    def _init_raw(self, data, t: FitTask, train: torch.Tensor, K: int) -> torch.Tensor:
        rp = t.params
        out = torch.zeros(K, dtype=torch.float64, device=data.device)
        if rp["init_zero"]:
            return out
        loss = rp["loss"]
        if getattr(data, "is_row_shard", False):   # global class priors / mean from summed counts
            if loss in (LOSS_LOG, LOSS_EXP):
                yc = data.y_cls[train].long()
                cnt = data.all_reduce(torch.bincount(yc, minlength=max(2, K)).double())
                pr = cnt / cnt.sum().clamp_min(1)
                if K == 1:
                    p = float(pr[1].clamp(_F32_EPS, 1 - _F32_EPS))
                    logit = math.log(p / (1 - p))
                    out[0] = logit if loss == LOSS_LOG else 0.5 * logit
                else:
                    lp = pr.clamp(_F32_EPS, 1 - _F32_EPS).log()
                    out[:] = lp - lp.mean()
                return out
            y = data.y_reg[train].double()
            if loss in (LOSS_ABS, LOSS_HUBER, LOSS_QUANT):   # percentile of the global training targets
                cnt = data.all_gather_equal(torch.tensor([int(y.numel())], device=y.device)).cpu().numpy()
                out[0] = _percentile_linear(data._gather_rows(y, cnt), 0.5 if loss != LOSS_QUANT else rp["alpha"])
                return out
            acc = data.all_reduce(torch.stack([y.sum(), torch.tensor(float(y.numel()), dtype=torch.float64,
                                                                     device=y.device)]))
            out[0] = acc[0] / acc[1].clamp_min(1)
            return out
        if loss in (LOSS_LOG, LOSS_EXP):
            yc = data.y_cls[train].long()
            if K == 1:
                p = float((yc == 1).double().mean().clamp(_F32_EPS, 1 - _F32_EPS))
                logit = math.log(p / (1 - p))
                out[0] = logit if loss == LOSS_LOG else 0.5 * logit
            else:
                pr = torch.bincount(yc, minlength=K).double() / max(1, yc.numel())
                lp = pr.clamp(_F32_EPS, 1 - _F32_EPS).log()
                out[:] = lp - lp.mean()
            return out
        y = data.y_reg[train].double()
        if loss == LOSS_SQ:
            # correctly rounded mean (math.fsum) -- the same double on every device, so a
            # squared-error ensemble is the same on the GPU as on the host builder
            out[0] = math.fsum(y.cpu().numpy().tolist()) / max(1, y.numel())
        elif loss in (LOSS_ABS, LOSS_HUBER):
            out[0] = _percentile_linear(y, 0.5)
        else:
            out[0] = _percentile_linear(y, rp["alpha"])
        return out

    def _boost(self, data, batch: List[FitTask], K: int, keep_models: bool,
               follow: Optional[Dict[int, List[FitTask]]] = None) -> List[FitOutput]:
        t0 = time.perf_counter()
        # prefix fits (prefix_groups): raw scores of leader f after its first m stages
        follow = follow or {}
        checkpoints: Dict[int, Dict[int, List[FitTask]]] = {}
        for f, t in enumerate(batch):
            for fo in follow.get(t.task_id, []):
                checkpoints.setdefault(f, {}).setdefault(fo.params["n_estimators"], []).append(fo)
        keep_fit = [t.keep or any(fo.keep for fo in follow.get(t.task_id, [])) for t in batch]
        snaps: List[Any] = []
        dev, n, gpu = data.device, data.n, data.is_gpu
        F = len(batch)
        Xb = data.binned()
        Xb_host = None if gpu else Xb.numpy()
        split_idx = torch.tensor([t.split for t in batch], device=dev)
        train = data.roles[split_idx] == 1                                  # [F, n]
        clf = data.classification
        sharded = getattr(data, "is_row_shard", False)
        if sharded:
            # the held-out early-stopping split is not a sum over ranks; leaf percentiles are,
            # as byte histograms of the fused stage's radix select (GPU only)
            bad = [t for t in batch if t.params.get("n_iter_no_change") or
                   (t.params["loss"] in (LOSS_ABS, LOSS_HUBER, LOSS_QUANT) and not (gpu and sharded_pct_ok()))]
            if bad:
                raise ParamError("row-sharded GradientBoosting supports squared_error, log_loss and exponential "
                                 "losses (and, on GPU, absolute_error / huber / quantile) without "
                                 "n_iter_no_change; run this job task-parallel")
        # early stopping (n_iter_no_change): sklearn holds out validation_fraction of the
        # fit's training rows (train_test_split, stratified for classifiers, seeded by
        # random_state) and stops when the validation loss has not improved by tol over
        # the last n_iter_no_change stages; the stage that triggers the stop is kept
        val_rows: Dict[int, torch.Tensor] = {}
        hist: Dict[int, np.ndarray] = {}
        for f, t in enumerate(batch):
            nic = t.params.get("n_iter_no_change")
            if not nic:
                continue
            tr = torch.nonzero(train[f]).squeeze(1).cpu().numpy()
            rs = t.params.get("random_state_int")
            rs = rs if rs is not None else int(t.seed) & 0x7FFFFFFF
            if clf:
                _, va = cv_mod.stratified_holdout_indices(data.y_enc[tr], t.params["validation_fraction"], rs)
            else:
                _, va = cv_mod.holdout_indices(len(tr), t.params["validation_fraction"], rs)
            vr = torch.from_numpy(tr[np.sort(va)]).to(dev)
            train[f, vr] = False
            val_rows[f] = vr
            hist[f] = np.full(int(nic), np.inf)
        if clf:
            ycls = data.y_cls.long()
            Y = torch.nn.functional.one_hot(ycls, max(2, data.n_classes)).double().t()   # [C, n]
            ybin = Y[1]
        else:
            yreg = data.y_reg.double()
        raw = torch.stack([self._init_raw(data, t, train[f], K) for f, t in enumerate(batch)])   # [F, K]
        init = raw.clone()
        raw = raw[:, :, None].repeat(1, 1, n).contiguous()                 # [F, K, n]
        lr = torch.tensor([t.params["learning_rate"] for t in batch], dtype=torch.float64, device=dev)
        n_est = [t.params["n_estimators"] for t in batch]
        seeds = [t.params["seed"] if t.params["seed"] is not None else t.seed for t in batch]
        gens = [torch.Generator(device="cpu").manual_seed(int(s) & 0x7FFFFFFF) for s in seeds]
        kept: List[List[Any]] = [[] for _ in range(F)]
        train_idx = [torch.nonzero(train[f]).squeeze(1) for f in range(F)]
        # fused HIP stage (csrc/kernels/gbrt.hip): gradient, leaf line search and raw update as
        # three kernels per stage instead of torch glue (losses with sums-only line searches)
        # percentile losses (absolute_error / huber / quantile) run fused too: leaf percentiles and
        # huber's delta by the exact radix select of gbrt.hip (early stopping reads the stage's
        # delta from the device for huber's validation loss)
        pct = (LOSS_ABS, LOSS_HUBER, LOSS_QUANT)
        # row-sharded stages run the same kernels in phases, with the leaf sums and the select
        # counters all-reduced between them (_sharded_stage)
        fused = (gpu and os.environ.get("DML_GB_FUSED", "1") != "0" and K <= 64
                 and all(t.params["loss"] in (LOSS_SQ, LOSS_LOG, LOSS_EXP) or
                         (t.params["loss"] in pct and not clf)
                         for t in batch)
                 and max(t.params["max_depth"] for t in batch) <= 10   # gbrt.hip: S <= 2048 path slots
                 and getattr(native.hip_lib(), "dml_gb_stage", None) is not None
                 and (not sharded or sharded_pct_ok()))
        if sharded and not fused and any(t.params["loss"] in pct for t in batch):
            raise ParamError("row-sharded GradientBoosting with absolute_error / huber / quantile losses needs "
                             "the fused GPU stage (max_depth <= 10); run this job task-parallel")
        if fused:
            lib = native.hip_lib()
            stream = native.stream_handle(dev)
            S = max(4, 2 ** (max(t.params["max_depth"] for t in batch) + 1))   # leaf path slots per tree
            G64 = torch.empty((F * K, n), dtype=torch.float64, device=dev)
            T32 = torch.empty((F * K, n), dtype=torch.float32, device=dev)
            ycls32 = data.y_cls.to(torch.int32).contiguous() if clf else torch.zeros(1, dtype=torch.int32, device=dev)
            yreg64 = torch.zeros(1, dtype=torch.float64, device=dev) if clf else yreg.contiguous()
            loss_all = np.array([t.params["loss"] for t in batch], dtype=np.int32)   # LOSS_* == gbrt.hip GbLoss
            lr_all = np.array([t.params["learning_rate"] for t in batch], dtype=np.float64)
            pct_any = bool(np.isin(loss_all, pct).any())
            alpha_all = np.array([float(t.params.get("alpha", 0.9)) for t in batch], dtype=np.float64)
            if pct_any:   # select scratch: leaf slot per (tree, row), byte counters (kept zero), states
                slot_of = torch.empty((F * K, n), dtype=torch.int16, device=dev)
                sel_hist = torch.zeros(max(F * K * S, F) * 256, dtype=torch.int32, device=dev)
                sel_state = torch.empty(max(F * K * S, F) * 4, dtype=torch.int64, device=dev)
                fit_delta = torch.zeros(F, dtype=torch.float64, device=dev)
            # per-stage leaf tables, allocated once at the batch's size and sliced per stage (a fresh
            # allocation per active-set size cost ~1 ms of allocator time before the stage kernels)
            slot_sum_all = torch.empty((F * K, S, 2), dtype=torch.float64, device=dev)
            slot_node_all = torch.empty((F * K, S), dtype=torch.int32, device=dev)
            slot_val_all = torch.empty((F * K, S), dtype=torch.float64, device=dev)
        if sharded:   # the global training rows (ascending), for subsample draws equal on every rank
            cnts = [data.all_gather_equal(torch.tensor([int(ti.numel())], device=dev)).cpu().numpy() for ti in train_idx]
            gtrain = [data._gather_rows(ti + data.r0, c) for ti, c in zip(train_idx, cnts)]
        # per-active-set device constants, made once: a pageable host->device copy per stage
        # waits for the stream, i.e. for the previous stage's kernels, before the next stage's
        # launches are even issued (the active set only changes when a fit stops)
        consts: Dict[tuple, Dict[str, Any]] = {}
        for stage in range(max(n_est)):
            act = [f for f in range(F) if stage < n_est[f]]
            if not act:
                break
            A = len(act)
            cst = consts.get(tuple(act))
            if cst is None:
                consts.clear()
                cst = consts[tuple(act)] = {"act_t": torch.tensor(act, device=dev)}
                if fused:
                    act_np = np.asarray(act, dtype=np.int32)
                    j_fit = np.repeat(act_np, K)
                    cst["fit_raw"] = torch.from_numpy(act_np * K).to(dev)
                    cst["fit_loss"] = torch.from_numpy(loss_all[act_np]).to(dev)
                    cst["tree_raw"] = torch.from_numpy(j_fit * K + np.tile(np.arange(K, dtype=np.int32), A)).to(dev)
                    cst["tree_loss"] = torch.from_numpy(loss_all[j_fit]).to(dev)
                    cst["tree_lr"] = torch.from_numpy(lr_all[j_fit]).to(dev)
                    if pct_any:
                        cst["fit_alpha"] = torch.from_numpy(alpha_all[act_np]).to(dev)
                        cst["tree_q"] = torch.from_numpy(np.where(loss_all[j_fit] == LOSS_QUANT, alpha_all[j_fit],
                                                                  0.5)).to(dev)
                        cst["fit_train"] = train[torch.from_numpy(act_np).to(dev).long()].to(torch.uint8).contiguous()
            act_t = cst["act_t"]
            loss = [batch[f].params["loss"] for f in act]
            hub_delta: Dict[int, float] = {}
            if fused:   # --- negative gradient of every active fit: one kernel -------------------
                fit_raw, fit_loss = cst["fit_raw"], cst["fit_loss"]
                ga = native.GbGradArgs(n=n, K=K, A=A, fit_raw=native.ptr(fit_raw), fit_loss=native.ptr(fit_loss),
                                       raw=native.ptr(raw), ycls=native.ptr(ycls32), yreg=native.ptr(yreg64),
                                       grad=native.ptr(G64), tgt=native.ptr(T32))
                if pct_any:
                    ga.fit_alpha, ga.fit_delta = native.ptr(cst["fit_alpha"]), native.ptr(fit_delta)
                    ga.fit_train, ga.sel_hist, ga.sel_state = (native.ptr(cst["fit_train"]), native.ptr(sel_hist),
                                                               native.ptr(sel_state))
                    if LOSS_HUBER in loss_all[act]:   # delta = alpha percentile of |y - raw| over training rows
                        if sharded:   # byte counts summed over the ranks' rows between passes
                            _radix_select(lib.dml_gb_fit_sel_step, ga, stream, data, sel_hist[:A * 256], 3)
                        else:
                            rc = lib.dml_gb_huber_delta(ctypes.byref(ga), stream)
                            if rc:
                                raise RuntimeError(f"dml_gb_huber_delta failed ({rc})")
                        for a, f in enumerate(act):   # early stopping: the stage's delta (read lazily)
                            if f in val_rows and loss_all[f] == LOSS_HUBER:
                                hub_delta[f] = fit_delta[a].clone()
                rc = lib.dml_gb_grad(ctypes.byref(ga), stream)
                if rc:
                    raise RuntimeError(f"dml_gb_grad failed ({rc})")
            else:
                R = raw[act_t]                                             # [A, K, n]
                # --- negative gradient (pseudo-residuals) --------------------------------
                G = torch.empty_like(R)
                for a, f in enumerate(act):
                    G[a], hub_delta[f] = self._neg_grad(batch[f].params, R[a], Y if clf else None,
                                                        ybin if clf else None, None if clf else yreg, K, train[f])
            # --- in-bag rows: the split's train rows, or a per-stage subsample of them ---
            inbag = train[act_t]
            sub_rows = []
            for a, f in enumerate(act):
                sub = batch[f].params["subsample"]
                if sub < 1.0:
                    tr = gtrain[f] if sharded else train_idx[f]
                    m = max(1, int(sub * tr.numel()))
                    pick = torch.randperm(tr.numel(), generator=gens[f])[:m].to(dev)
                    row = torch.zeros(n, dtype=torch.bool, device=dev)
                    sel = tr[pick]
                    if sharded:   # this rank's share of the global draw
                        sel = sel - data.r0
                        sel = sel[(sel >= 0) & (sel < n)]
                    row[sel] = True
                    inbag[a] = row
                    sub_rows.append(a)
            # one role row per tree (roles = in-bag mask of its fit); fixed while the active set
            # is, unless a fit subsamples
            J = A * K
            roles_t = cst.get("roles_t") if not sub_rows else None
            if roles_t is None:
                roles_t = inbag.repeat_interleave(K, dim=0).to(torch.uint8).contiguous()   # [J, n]
                if not sub_rows:
                    cst["roles_t"] = roles_t
            tgt = T32[:J] if fused else G.reshape(J, n).float().contiguous()
            specs = _stage_specs(batch, act, K, seeds, stage)
            limit = np.repeat([batch[f].params.get("max_leaf_nodes", 0) for f in act], K)
            ccp = np.repeat([batch[f].params.get("ccp_alpha", 0.0) for f in act], K)
            if sharded:   # level-synchronous trees over the row shards (ops/forest_dp.py)
                from ..ops import forest_dp

                fb = forest_dp.build_dp(Xb, None, tgt, roles_t, specs, 1, True, data.r0, reduce=data.all_reduce,
                                        comm=data, ystride=n)
                if not gpu:
                    fb = fb.to_numpy()
                if limit.any():
                    forest_ops.prune_max_leaves(fb, specs, limit)
                if ccp.any():
                    forest_ops.prune_ccp(fb, specs, ccp)
                bv, ex = data.bin_values()
                if bool(ex.any()):
                    nodes_t = fb.nodes if gpu else torch.from_numpy(fb.nodes)
                    fbt = forest_ops.ForestBuild(nodes_t, fb.vals, fb.n_trees, fb.VC, True, 1)
                    forest_dp.refine_dp(fbt, Xb, roles_t, specs, data.r0, bv, ex, reduce=data.all_reduce)
                xbt = None
                if fused:   # the fused stage walks the trees itself
                    leaf = None
                else:
                    leaf = (forest_ops.apply(fb, Xb).long() if gpu
                            else torch.from_numpy(forest_ops.apply(fb, Xb_host)).long())
                vals = fb.vals if gpu else torch.from_numpy(fb.vals)
            elif gpu:
                # feature-major bins: the large tier's gathers of a dense sorted row set coalesce
                # (64 rows of one feature in 1-2 cache lines instead of 64 row lines)
                xbt = data.binned_feature_major() if hasattr(data, "binned_feature_major") else None
                # per-tree active-row counts: fixed while the roles are (no subsample draw)
                ccache = cst.setdefault("count_cache", {}) if not sub_rows else None
                # the roots' row-count histograms are fixed while the roles are (DML_GB_ROOT_CACHE=0: off)
                rcache = (cst.setdefault("root_counts", {})
                          if not sub_rows and os.environ.get("DML_GB_ROOT_CACHE", "1") != "0" else None)
                fb = forest_ops.build_gpu(Xb, None, tgt, roles_t, specs, 1, True, self.tiers, ystride=n, XbT=xbt,
                                          count_cache=ccache, root_counts=rcache)
                if limit.any():   # sklearn's best-first tree (friedman_mse and squared_error rank splits alike)
                    forest_ops.prune_max_leaves(fb, specs, limit)
                if ccp.any():     # minimal cost-complexity pruning of each stage tree (variance impurity)
                    forest_ops.prune_ccp(fb, specs, ccp)
                _refine(data, fb, Xb, specs, roles_t)
                leaf = None if fused else forest_ops.apply(fb, Xb).long()  # [J, n] (the fused stage walks itself)
                vals = fb.vals
            else:
                fb = forest_ops.build_cpu(Xb_host, None, tgt.numpy(), roles_t.numpy(), specs, 1, True, ystride=n)
                if limit.any():
                    forest_ops.prune_max_leaves(fb, specs, limit)
                if ccp.any():
                    forest_ops.prune_ccp(fb, specs, ccp)
                _refine(data, fb, Xb, specs, roles_t)
                leaf = torch.from_numpy(forest_ops.apply(fb, Xb_host)).long()
                vals = torch.from_numpy(fb.vals)
            P = vals.shape[0]
            if fused:   # --- leaf line search + raw update of every row: three kernels ------------
                tree_raw, tree_loss, tree_lr = cst["tree_raw"], cst["tree_loss"], cst["tree_lr"]
                slot_sum, slot_node, slot_val = slot_sum_all[:J].zero_(), slot_node_all[:J].fill_(-1), slot_val_all[:J]
                sa = native.GbStageArgs(Xb=native.ptr(Xb), ld=Xb.stride(0), n=n, nodes=native.ptr(fb.nodes),
                                        node_val=native.ptr(vals), J=J, K=K, S=S, tree_raw=native.ptr(tree_raw),
                                        tree_loss=native.ptr(tree_loss), tree_lr=native.ptr(tree_lr),
                                        inbag=native.ptr(roles_t), grad=native.ptr(G64), ycls=native.ptr(ycls32),
                                        slot_sum=native.ptr(slot_sum), slot_node=native.ptr(slot_node),
                                        slot_val=native.ptr(slot_val), raw=native.ptr(raw),
                                        XbT=native.ptr(xbt) if xbt is not None else 0)
                if pct_any:
                    sa.pct_any, sa.yreg, sa.slot_of = 1, native.ptr(yreg64), native.ptr(slot_of)
                    sa.sel_hist, sa.sel_state = native.ptr(sel_hist), native.ptr(sel_state)
                    sa.tree_q, sa.tree_delta = native.ptr(cst["tree_q"]), native.ptr(fit_delta)
                if sharded:
                    _sharded_stage(lib, sa, stream, data, slot_sum, sel_hist[:J * S * 256] if pct_any else None,
                                   newton=bool(np.isin(loss_all[act], (LOSS_LOG, LOSS_EXP)).any()),
                                   huber=LOSS_HUBER in loss_all[act])
                else:
                    rc = lib.dml_gb_stage(ctypes.byref(sa), stream)
                    if rc:
                        raise RuntimeError(f"dml_gb_stage failed ({rc})")
                if keep_models:   # node-indexed leaf values for the kept trees
                    value = torch.zeros(P, dtype=torch.float64, device=dev)
                    ok = slot_node >= 0
                    value[slot_node[ok].long()] = slot_val[ok]
            else:
                value = self._line_search(batch, act, loss, vals, leaf_of=lambda: leaf, roles_t=roles_t, G=G, R=R,
                                          Y=Y if clf else None, ybin=ybin if clf else None,
                                          yreg=None if clf else yreg, K=K, J=J, n=n, P=P, hub_delta=hub_delta,
                                          sharded=sharded, data=data)
                # --- raw-score update of every row (train and held-out) --------------------
                upd = value[leaf].view(A, K, n) * lr[act_t].view(A, 1, 1)
                raw[act_t] += upd
            for a, f in enumerate(act):
                if f in val_rows:
                    vl = self._val_loss(batch[f].params, raw[f][:, val_rows[f]], val_rows[f], data, K, hub_delta.get(f))
                    h = hist[f]
                    if np.any(vl + batch[f].params["tol"] < h):
                        h[stage % len(h)] = vl
                    else:
                        n_est[f] = stage + 1     # this stage is the fit's last (sklearn keeps it)
            if keep_models:
                vals_np = value.cpu().numpy()
                nodes_np = fb.nodes.cpu().numpy() if isinstance(fb.nodes, torch.Tensor) else fb.nodes
                for a, f in enumerate(act):
                    if not keep_fit[f]:
                        continue
                    lr_f = float(lr[f])
                    kept[f].append([_extract_tree(nodes_np, vals_np * lr_f, a * K + k) for k in range(K)])
            for f in act:   # prefix fits that end at this stage
                for fo in checkpoints.get(f, {}).get(stage + 1, []):
                    snaps.append((fo, f, raw[f].clone()))
        if gpu:
            torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        outs = self._outputs(batch, raw, init, kept, data, K, clf, keep_models, dt)
        if snaps:
            outs += self._outputs([s[0] for s in snaps], torch.stack([s[2] for s in snaps]),
                                  torch.stack([init[s[1]] for s in snaps]),
                                  [kept[s[1]][:s[0].params["n_estimators"]] for s in snaps], data, K, clf,
                                  keep_models, dt)
        return outs

    @staticmethod
    def _line_search(batch, act, loss, vals, leaf_of, roles_t, G, R, Y, ybin, yreg, K, J, n, P, hub_delta, sharded,
                     data):
        """Leaf values of one stage (torch path): node means for squared error, one Newton
        step for log-loss / exponential, (weighted) percentiles for absolute / huber / quantile."""
        dev = vals.device
        leaf = leaf_of()
        # --- leaf values (line search) -----------------------------------------------
        value = vals[:, 1] / vals[:, 0].clamp_min(1e-300)             # squared error: node mean
        value = torch.where(vals[:, 0] > 0, value, torch.zeros_like(value))
        m = roles_t.bool()
        lf = leaf[m]
        needs = {l for l in loss if l != LOSS_SQ}
        if needs:
            value = value.clone()
            tree_of = torch.arange(J, device=dev).view(J, 1).expand(J, n)[m]
            fit_of_tree = torch.tensor([act[j // K] for j in range(J)], device=dev)
            loss_of_tree = torch.tensor([loss[j // K] for j in range(J)], device=dev)
            g = G.reshape(J, n)[m]
            node_loss = torch.full((P,), -1, dtype=torch.long, device=dev)
            node_loss.scatter_(0, lf, loss_of_tree[tree_of])
            if LOSS_LOG in needs or LOSS_EXP in needs:
                num = leaf_sum(lf, g, P)
                if K > 1:
                    yk = Y[torch.arange(J, device=dev) % K].reshape(J, n)[m]
                    prob = yk - g
                    hess = prob * (1 - prob)
                    num = num * (K - 1) / K
                else:
                    yb = ybin.view(1, n).expand(J, n)[m]
                    prob = yb - g
                    hess_log = prob * (1 - prob)
                    hess_exp = torch.where(yb > 0.5, g, -g)
                    is_exp = loss_of_tree[tree_of] == LOSS_EXP
                    hess = torch.where(is_exp, hess_exp, hess_log)
                den = leaf_sum(lf, hess, P)
                if sharded:   # leaf sums over every rank's rows
                    num, den = data.all_reduce(num), data.all_reduce(den)
                newton = torch.where(den.abs() < 1e-150, torch.where(num == 0, 0.0, torch.sign(num) * 1e150),
                                     num / torch.where(den.abs() < 1e-150, torch.ones_like(den), den))
                sel = (node_loss == LOSS_LOG) | (node_loss == LOSS_EXP)
                value = torch.where(sel, newton, value)
            if needs & {LOSS_ABS, LOSS_HUBER, LOSS_QUANT}:
                resid = (yreg.view(1, n) - R.reshape(J, n))[m]        # y - raw (K == 1 for regression)
                for lk in needs & {LOSS_ABS, LOSS_HUBER, LOSS_QUANT}:
                    sel_rows = loss_of_tree[tree_of] == lk
                    if lk == LOSS_QUANT:
                        # per-tree alpha: group trees by alpha
                        for alpha in sorted({batch[act[j // K]].params["alpha"] for j in range(J)
                                             if loss[j // K] == lk}):
                            trees = torch.tensor([j for j in range(J) if loss[j // K] == lk and
                                                  batch[act[j // K]].params["alpha"] == alpha], device=dev)
                            rs = sel_rows & torch.isin(tree_of, trees)
                            pv = _segment_percentile(lf[rs], resid[rs], P, alpha)
                            value = torch.where(~torch.isnan(pv), pv, value)
                        continue
                    med = _segment_percentile(lf[sel_rows], resid[sel_rows], P, 0.5)
                    if lk == LOSS_ABS:
                        value = torch.where(~torch.isnan(med), med, value)
                    else:
                        delta = torch.zeros(J, dtype=torch.float64, device=dev)
                        for j in range(J):
                            if loss[j // K] == LOSS_HUBER:
                                delta[j] = hub_delta[act[j // K]]
                        diff = resid[sel_rows] - med[lf[sel_rows]]
                        dl = delta[tree_of[sel_rows]]
                        term = torch.sign(diff) * torch.minimum(dl, diff.abs())
                        s_ = leaf_sum(lf[sel_rows], term, P)
                        c_ = torch.bincount(lf[sel_rows], minlength=P).to(torch.float64)
                        hub = med + s_ / c_.clamp_min(1)
                        value = torch.where(~torch.isnan(med), hub, value)
        return value

    @staticmethod
    def _outputs(batch, raw, init, kept, data, K, clf, keep_models, dt) -> List[FitOutput]:
        F = len(batch)
        outs = []
        for f, t in enumerate(batch):
            rows = data.test_rows[t.split].long()
            r = raw[f][:, rows]                                            # [K, m]
            lossf = t.params["loss"]
            proba = None
            if not clf:
                pred = r[0].float()
            elif K == 1:
                z = 2 * r[0] if lossf == LOSS_EXP else r[0]
                p1 = torch.sigmoid(z)
                proba = torch.stack([1 - p1, p1], 1)
                pred = (r[0] >= 0).to(torch.int32)
            else:
                proba = torch.softmax(r.t(), 1)
                pred = r.argmax(0).to(torch.int32)
            o = FitOutput(task_id=t.task_id, pred=pred, proba=proba, fit_seconds=dt / F,
                          info={"warnings": t.params.get("warnings", [])})
            if keep_models and t.keep:
                o.model = _pack_model(kept[f], init[f].cpu().numpy(), t, data, K)
            outs.append(o)
        return outs

    @staticmethod
    def _val_loss(rp, r, rows, data, K, delta) -> float:
        """sklearn's ``self._loss(y_val, raw_val)``: mean of the half-losses GradientBoosting
        uses (HalfBinomial / HalfMultinomial / Exponential / HalfSquared / Absolute / Pinball /
        Huber at the stage's delta) over the validation rows."""
        loss = rp["loss"]
        if loss in (LOSS_LOG, LOSS_EXP):
            y = data.y_cls[rows].long()
            if loss == LOSS_EXP:
                return float(torch.exp(-(2.0 * y.double() - 1.0) * r[0]).mean())
            if K == 1:
                z = r[0]
                return float((torch.nn.functional.softplus(z) - y.double() * z).mean())
            return float((torch.logsumexp(r, 0) - r.gather(0, y.view(1, -1))[0]).mean())
        d = data.y_reg[rows].double() - r[0]
        if loss == LOSS_SQ:
            return float((0.5 * d * d).mean())
        if loss == LOSS_ABS:
            return float(d.abs().mean())
        if loss == LOSS_QUANT:
            a = rp["alpha"]
            return float(torch.where(d >= 0, a * d, (a - 1.0) * d).mean())
        dl = float(delta or 0.0)
        ad = d.abs()
        return float(torch.where(ad <= dl, 0.5 * d * d, dl * (ad - 0.5 * dl)).mean())

    # negative gradient [K, n] of the fit's loss (+ huber delta, else 0)
    @staticmethod
    def _neg_grad(rp, r, Y, ybin, yreg, K, train_row):
        loss = rp["loss"]
        if loss == LOSS_LOG:
            if K == 1:
                return (ybin - torch.sigmoid(r[0])).view(1, -1), 0.0
            return Y[:K] - torch.softmax(r, 0), 0.0
        if loss == LOSS_EXP:
            return (ybin * torch.exp(-r[0]) - (1 - ybin) * torch.exp(r[0])).view(1, -1), 0.0
        diff = yreg - r[0]
        if loss == LOSS_SQ:
            return diff.view(1, -1), 0.0
        if loss == LOSS_ABS:
            return torch.sign(diff).view(1, -1), 0.0
        if loss == LOSS_QUANT:
            a = rp["alpha"]
            return torch.where(diff >= 0, torch.full_like(diff, a), torch.full_like(diff, a - 1)).view(1, -1), 0.0
        # huber: delta = alpha-percentile of |y - raw| over the fit's training rows (set_huber_delta)
        delta = float(_percentile_icdf(diff[train_row].abs(), rp["alpha"]))
        return torch.where(diff.abs() <= delta, diff, delta * torch.sign(diff)).view(1, -1), delta


def _stage_specs(batch, act: List[int], K: int, seeds: List[int], stage: int) -> np.ndarray:
    """TreeSpecs of one stage: tree j = a * K + k grows fit act[a]'s class-k tree on target
    row j with in-bag role row j (built column-wise, not field by field per tree)."""
    A = len(act)
    J = A * K
    specs = forest_ops.make_specs(J)
    if J == 0:
        return specs
    rps = [batch[f].params for f in act]
    rep = lambda vals, dt: np.repeat(np.asarray(vals, dtype=dt), K)
    specs["seed"] = [native_seed(seeds[f], stage * K + k) for f in act for k in range(K)]
    j = np.arange(J, dtype=np.int32)
    specs["split"] = j
    specs["fit"] = j
    specs["target"] = j
    specs["max_depth"] = rep([rp["max_depth"] for rp in rps], np.int64)
    specs["min_samples_split"] = rep([rp["min_samples_split"] for rp in rps], np.int64)
    specs["min_samples_leaf"] = rep([rp["min_samples_leaf"] for rp in rps], np.int64)
    specs["max_features"] = rep([rp["max_features"] for rp in rps], np.int64)
    specs["bootstrap"] = 0
    specs["criterion"] = rep([rp.get("criterion", forest_ops.MSE) for rp in rps], np.int64)
    specs["min_impurity_decrease"] = rep([rp["min_impurity_decrease"] for rp in rps], np.float64)
    specs["min_weight_frac"] = rep([rp.get("min_weight_fraction_leaf", 0.0) for rp in rps], np.float64)
    return specs


def _extract_tree(nodes: np.ndarray, values: np.ndarray, root: int):
    """Standalone (nodes [m,2], value [m]) of the tree rooted at ``root`` (root first)."""
    ids = {root: 0}
    order = [root]
    out_nodes, out_vals = [], []
    i = 0
    while i < len(order):
        nd = order[i]
        sp, left = int(nodes[nd, 0]), int(nodes[nd, 1])
        if sp >= 0:
            ids[left], ids[left + 1] = len(order), len(order) + 1
            order.extend([left, left + 1])
        i += 1
    for nd in order:
        sp, left = int(nodes[nd, 0]), int(nodes[nd, 1])
        out_nodes.append((sp, ids[left] if sp >= 0 else -1))
        out_vals.append(float(values[nd]))
    return np.asarray(out_nodes, dtype=np.int32), np.asarray(out_vals, dtype=np.float64)


def leaf_sum(leaf: torch.Tensor, v: torch.Tensor, P: int) -> torch.Tensor:
    """Per-leaf float64 sums of ``v`` (leaf ids in [0, P)).  A plain ``index_add_`` sends a
    whole stage's rows -- fits x trees x 800k -- into the few leaves of depth-3..5 trees:
    every add hits one of a handful of addresses and the float64 atomics serialise (82 of
    88 s of the config-6 GBRT grid, profiles/r3_gbrt_config6.md).  Here each row
    adds into its own copy of the leaf vector (C x P addresses, rows interleaved over the
    copies), and the copies are summed."""
    n = int(leaf.numel())
    if n == 0:
        return torch.zeros(P, dtype=torch.float64, device=v.device)
    C = int(max(1, min(n // 4096, 1024, (64 << 20) // max(1, P))))
    if C == 1:
        return torch.zeros(P, dtype=torch.float64, device=v.device).index_add_(0, leaf, v.to(torch.float64))
    # interleaved copies: consecutive rows (one tree, one or two leaves) go to different
    # copies, so a wave's 64 adds land on 64 addresses instead of queueing on one
    chunk = torch.arange(n, device=leaf.device, dtype=torch.int64) % C
    part = torch.zeros(C * P, dtype=torch.float64, device=v.device)
    part.index_add_(0, chunk * P + leaf.to(torch.int64), v.to(torch.float64))
    return part.view(C, P).sum(0)


def _pack_model(stages, init: np.ndarray, t: FitTask, data, K: int) -> Dict[str, Any]:
    nodes, vals, roots = [], [], []
    off = 0
    for st in stages:
        rr = []
        for nd, vv in st:
            nd = nd.copy()
            nd[:, 1] = np.where(nd[:, 1] >= 0, nd[:, 1] + off, -1)
            nodes.append(nd)
            vals.append(vv)
            rr.append(off)
            off += len(nd)
        roots.append(rr)
    return {
        "kind": "gbrt", "nodes": np.concatenate(nodes) if nodes else np.zeros((0, 2), np.int32),
        "value": np.concatenate(vals) if vals else np.zeros(0), "roots": np.asarray(roots, dtype=np.int32),
        "init": init, "K": K, "loss": int(t.params["loss"]), "edges": data.edges.cpu().numpy(),
        "classes": None if data.classes is None else np.asarray(data.classes).tolist(),
        "model_type": t.model_type, "params": {k: v for k, v in t.params.items() if k != "warnings"},
    }


def gbrt_raw_numpy(model: Dict[str, Any], X: np.ndarray) -> np.ndarray:
    lib = native.cpu_lib()
    X = np.ascontiguousarray(X, dtype=np.float32)
    edges = np.ascontiguousarray(model["edges"], dtype=np.float32)
    Xb = np.empty(X.shape, dtype=np.uint8)
    lib.dml_cpu_bin(native.ptr(X), X.shape[0], X.shape[1], native.ptr(edges), native.ptr(Xb), X.shape[1])
    nodes, value, roots = model["nodes"], model["value"], np.asarray(model["roots"])
    K = int(model["K"])
    raw = np.tile(np.asarray(model["init"], dtype=np.float64), (X.shape[0], 1))
    rows = np.arange(X.shape[0])
    for s in range(roots.shape[0]):
        for k in range(K):
            node = np.full(X.shape[0], roots[s, k], dtype=np.int64)
            while True:
                sp = nodes[node, 0]
                inner = sp >= 0
                if not inner.any():
                    break
                feat, b = np.where(inner, sp >> 8, 0), np.where(inner, sp & 255, 0)
                go = Xb[rows, feat] > b
                node = np.where(inner, nodes[node, 1] + go, node)
            raw[:, k] += value[node]
    return raw


def gbrt_predict_numpy(model: Dict[str, Any], X: np.ndarray) -> np.ndarray:
    raw = gbrt_raw_numpy(model, X)
    if model.get("classes") is None:
        return raw[:, 0]
    idx = (raw[:, 0] >= 0).astype(int) if raw.shape[1] == 1 else raw.argmax(1)
    return np.asarray(model["classes"])[idx]


register(GradientBoostingFamily())
