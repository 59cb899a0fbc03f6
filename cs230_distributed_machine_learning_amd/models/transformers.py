"""Transformer estimators of the reference whitelist (aws-prod/worker/worker.py:52-56).

The reference lists ``StandardScaler``, ``MinMaxScaler``, ``PCA``, ``OneHotEncoder`` and
``SimpleImputer`` as trainable model types, but its worker cannot run them:
``check_model_type`` returns "Unknown model type" and the regressor branch then calls
``.predict`` on a transformer (worker.py:320-341, 458-468).

Here:

* ``PCA`` is a real searchable estimator, with sklearn's GridSearchCV semantics: with no
  ``scoring`` the CV score is ``PCA.score`` (mean log-likelihood of the held-out rows
  under the probabilistic-PCA model).  One covariance GEMM + symmetric eigendecomposition
  per split (on the device) serves EVERY candidate of that split: ``n_components`` (int,
  variance fraction, 'mle', None) and ``whiten`` only change how the spectrum is cut, so
  held-out log-likelihoods for all candidates come from one projection of the test rows
  onto the eigenbasis.
* The four column-wise transformers have no ``score``/``predict``; sklearn's
  GridSearchCV rejects them without a scorer, and so does this engine — with a message
  pointing at ``/preprocess`` (data/preprocess.py), which applies the same scaling /
  imputation / one-hot transforms to a dataset.
"""
from __future__ import annotations

import math
import os
import time
from typing import Any, Dict, List

import numpy as np
import torch

from .base import Family, FitOutput, FitTask, ParamError, as_bool, as_float, as_int, register

_PCA_DEFAULTS = {"n_components": None, "copy": True, "whiten": False, "svd_solver": "auto", "tol": 0.0,
                 "iterated_power": "auto", "n_oversamples": 10, "power_iteration_normalizer": "auto",
                 "random_state": None}
_EPS = float(np.finfo(np.float64).eps)


def _assess_dimension(spectrum: np.ndarray, rank: int, n_samples: int) -> float:
    """Minka (2000) log-likelihood of a rank-``rank`` PPCA model (sklearn PCA 'mle')."""
    from scipy.special import gammaln

    n_features = spectrum.shape[0]
    if spectrum[rank - 1] < 1e-15:
        return -math.inf
    pu = -rank * math.log(2.0)
    for i in range(1, rank + 1):
        pu += gammaln((n_features - i + 1) / 2.0) - math.log(math.pi) * (n_features - i + 1) / 2.0
    pl = -np.sum(np.log(spectrum[:rank])) * n_samples / 2.0
    v = max(_EPS, np.sum(spectrum[rank:]) / (n_features - rank))
    pv = -math.log(v) * n_samples * (n_features - rank) / 2.0
    m = n_features * rank - rank * (rank + 1.0) / 2.0
    pp = math.log(2.0 * math.pi) * (m + rank) / 2.0
    spectrum_ = spectrum.copy()
    spectrum_[rank:n_features] = v
    pa = 0.0
    for i in range(rank):
        for j in range(i + 1, len(spectrum)):
            pa += math.log((spectrum[i] - spectrum[j]) * (1.0 / spectrum_[j] - 1.0 / spectrum_[i])) + math.log(n_samples)
    return pu + pl + pv + pp - pa / 2.0 - rank * math.log(n_samples) / 2.0


def _n_components(spec, ev: np.ndarray, n_samples: int, d: int) -> int:
    kmax = min(n_samples, d)
    if spec is None:
        return kmax
    if spec == "mle":
        ll = np.full(len(ev), -np.inf)
        for r in range(1, len(ev)):
            ll[r] = _assess_dimension(ev, r, n_samples)
        return int(ll.argmax())
    if isinstance(spec, float) and 0 < spec < 1:
        ratio = ev / ev.sum()
        return int(np.searchsorted(np.cumsum(ratio), spec, side="right") + 1)
    return int(spec)


class PCAFamily(Family):
    model_types = ("PCA",)
    classifiers = ()
    self_scored = ("PCA",)
    data_parallel = True   # row-sharded: [count, sum x, X^T X] and the test log-likelihood sums all-reduced
    dp_when_few = False
    streams_rows = True    # binned-only tables: covariance and test projections over streamed host rows

    def resolve(self, model_type, params, n_train, n_features, n_classes) -> Dict[str, Any]:
        p = dict(_PCA_DEFAULTS)
        p.update({k: v for k, v in params.items() if k in _PCA_DEFAULTS})
        warn = []
        nc = p["n_components"]
        if nc not in (None, "mle"):
            if isinstance(nc, float) and not nc.is_integer():
                if not 0 < nc < 1:
                    raise ParamError("n_components float must be in (0, 1)")
            else:
                nc = as_int(nc, "n_components", lo=0, hi=min(n_train, n_features))
        elif nc == "mle" and n_train < n_features:
            raise ParamError("n_components='mle' is only supported if n_samples >= n_features")
        if p["svd_solver"] in ("randomized", "arpack", "covariance_eigh"):
            warn.append(f"svd_solver={p['svd_solver']!r}: exact eigendecomposition used")
        return {"n_components": nc, "whiten": as_bool(p["whiten"], "whiten"), "warnings": warn}

    def cost(self, model_type, rp, n_train, n_features, n_classes) -> float:
        return n_train * n_features * n_features * 2e-12 + 1e-3

    def run(self, data, tasks: List[FitTask], keep_models: bool = False) -> List[FitOutput]:
        t0 = time.perf_counter()
        X = data.X
        d = data.d
        eig: Dict[int, Any] = {}
        outs = []
        fused = {}
        streamed = X is None and getattr(data, "can_stream_rows", lambda: False)()
        if streamed or (data.is_gpu and not getattr(data, "is_row_shard", False)
                        and os.environ.get("DML_LINREG_KERNEL", "1") != "0"):
            # every split's covariance from one pass over X (the LinearRegression moments kernel,
            # or the streamed moments of a table whose float32 rows are not resident)
            from .linear import LinearRegressionFamily, streamed_split_moments

            splits = sorted({t.split for t in tasks})
            M, shift = (streamed_split_moments(data, splits) if streamed
                        else LinearRegressionFamily.split_moments(data, splits))
            for i, sp in enumerate(splits):
                cnt, Sx, XX = M[i][d, d], M[i][:d, d], M[i][:d, :d]
                dm = Sx / cnt.clamp_min(1)
                fused[sp] = (shift[:d] + dm, (XX - cnt * torch.outer(dm, dm)) / max(1.0, float(cnt) - 1), int(cnt))
        sharded = getattr(data, "is_row_shard", False)
        if streamed:
            # every split's eigenbasis first, then all test projections in ONE pass over the rows
            from .linear import streamed_test_many

            basis = {}
            for sp in sorted({t.split for t in tasks}):
                mean, cov, n = fused[sp]
                lam, V = torch.linalg.eigh(cov)
                basis[sp] = (mean, lam.flip(0).clamp_min(0), V.flip(1), n)
            sps = list(basis)
            Zs = streamed_test_many(data, [(sp, lambda Xt, mean=basis[sp][0], V=basis[sp][2]: (Xt - mean) @ V)
                                           for sp in sps])
            for sp, Z in zip(sps, Zs):
                mean, lam, V, n = basis[sp]
                if Z is None:
                    Z = torch.zeros((0, d), dtype=torch.float64, device=data.device)
                eig[sp] = (mean, lam, V, Z, n)
        for t in tasks:
            if t.split not in eig:
                if t.split in fused:
                    mean, cov, n = fused[t.split]
                elif sharded:   # global moments: one all-reduce of [count, sum x, X^T X] (float64)
                    Xt = X[data.train_rows[t.split].long()].double()
                    m = torch.cat([torch.tensor([float(Xt.shape[0])], dtype=torch.float64, device=X.device),
                                   Xt.sum(0), (Xt.t() @ Xt).flatten()])
                    data.all_reduce(m)
                    n = int(m[0])
                    mean = m[1:1 + d] / max(1, n)
                    cov = (m[1 + d:].view(d, d) - n * torch.outer(mean, mean)) / max(1, n - 1)
                else:
                    tr = data.train_rows[t.split].long()
                    Xt = X[tr].double()
                    mean = Xt.mean(0)
                    Xc = Xt - mean
                    n = Xt.shape[0]
                    cov = Xc.t() @ Xc / max(1, n - 1)
                lam, V = torch.linalg.eigh(cov)                       # ascending
                lam, V = lam.flip(0).clamp_min(0), V.flip(1)
                if streamed:
                    from .linear import streamed_test_rows

                    Z = streamed_test_rows(data, t.split, lambda Xt, mean=mean, V=V: (Xt - mean) @ V)
                    if Z is None:
                        Z = torch.zeros((0, d), dtype=torch.float64, device=data.device)
                else:
                    te = data.test_rows[t.split].long()
                    Z = (X[te].double() - mean) @ V                    # test rows in the eigenbasis
                eig[t.split] = (mean, lam, V, Z, n)
            mean, lam, V, Z, n = eig[t.split]
            ev = lam.cpu().numpy()[: min(n, d)]
            try:
                k = _n_components(t.params["n_components"], ev, n, d)
            except ValueError as e:
                outs.append(FitOutput(task_id=t.task_id, error=str(e)))
                continue
            kmax = min(n, d)
            noise = float(ev[k:kmax].mean()) if k < kmax else 0.0
            lam_d = lam.clone()
            if t.params["whiten"]:
                top = lam[:k] * torch.clamp(lam[:k] - noise, min=0) + noise
            else:
                top = torch.where(lam[:k] > noise, lam[:k], torch.full_like(lam[:k], noise))
            lam_d[:k] = top
            lam_d[k:] = noise
            if noise == 0.0 and k < d:
                score = -math.inf
            else:
                ll = -0.5 * ((Z * Z) / lam_d).sum(1) - 0.5 * (d * math.log(2 * math.pi) + torch.log(lam_d).sum())
                if sharded:   # mean over the GLOBAL held-out rows
                    acc = data.all_reduce(torch.stack([ll.sum(), torch.tensor(float(ll.numel()), dtype=ll.dtype,
                                                                              device=ll.device)]))
                    score = float(acc[0] / acc[1].clamp_min(1))
                else:
                    score = float(ll.mean())
            o = FitOutput(task_id=t.task_id, info={"score": score, "n_components": k,
                                                   "warnings": t.params["warnings"]})
            if keep_models:
                o.model = {"kind": "pca", "mean": mean.cpu().numpy(), "components": V[:, :k].t().cpu().numpy(),
                           "var": lam[:k].cpu().numpy(), "noise_variance": noise, "whiten": t.params["whiten"],
                           "model_type": "PCA"}
            outs.append(o)
        data.sync()
        dt = time.perf_counter() - t0
        for o in outs:
            o.fit_seconds = dt / max(1, len(outs))
        return outs


class ColumnTransformerFamily(Family):
    """Whitelisted column transformers: rejected for search with a pointer to /preprocess."""

    model_types = ("StandardScaler", "MinMaxScaler", "OneHotEncoder", "SimpleImputer")
    classifiers = ()

    def resolve(self, model_type, params, n_train, n_features, n_classes):
        raise ParamError(
            f"{model_type} is a transformer with no score or predict method, so it cannot be cross-validated "
            f"(sklearn GridSearchCV raises the same); apply it to the dataset with /preprocess instead")


def pca_transform_numpy(model: Dict[str, Any], X: np.ndarray) -> np.ndarray:
    Z = (np.asarray(X, dtype=np.float64) - model["mean"]) @ np.asarray(model["components"]).T
    if model.get("whiten"):
        Z = Z / np.sqrt(np.asarray(model["var"]))
    return Z


register(PCAFamily())
register(ColumnTransformerFamily())
