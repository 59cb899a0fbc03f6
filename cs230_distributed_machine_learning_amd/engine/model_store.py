"""Model artefacts: safe on-disk format + CPU/GPU prediction.

The reference pickles every fitted sklearn model into the worker's local
``./models/<subtask>_model.pkl`` (aws-prod/worker/worker.py:351-356) and the master
tries to ``send_file`` a path that only exists on the worker (D18).  Here artefacts
live in one shared model store as ``.npz`` (arrays + a JSON metadata string; loaded
with ``allow_pickle=False``, so downloading and loading a model executes nothing).

Kinds: ``forest`` (pool layout of ops/forest_ops.py + bin edges),
``linear_logistic``, ``linear_regression``, ``knn`` (training rows), ``gbrt`` (stage trees),
``svm`` (support vectors + dual coefficients per one-vs-one machine), ``pca`` (mean,
components, explained variances, noise variance).

``load_predictor(path)`` wraps an artefact in an estimator-like object (``predict``,
``predict_proba`` / ``decision_function`` for classifiers, ``score``, ``transform`` for
PCA) -- what the reference's pickled sklearn estimator gives its user after
``download_best_model`` (DistributedLibrary/src/distributed_ml/core.py:201-206,
aws-prod/worker/worker.py:351-356), without unpickling anything.
"""
from __future__ import annotations

import json
import os
import re
from typing import Any, Dict, Optional

import numpy as np

_ARRAY_KEYS = ("nodes", "vals", "edges", "coef", "intercept", "X", "y", "init", "stage_offsets", "scale", "mean",
               "components", "var", "min", "max", "value", "roots")


def save_model(model: Dict[str, Any], path: str) -> str:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    arrays = {k: np.asarray(v) for k, v in model.items() if k in _ARRAY_KEYS and v is not None}
    meta = {k: v for k, v in model.items() if k not in _ARRAY_KEYS}
    tmp = path + ".tmp.npz"
    np.savez(tmp, __meta__=np.array(json.dumps(meta, default=_jdefault)), **arrays)
    os.replace(tmp, path)
    return path


def _jdefault(o):
    if isinstance(o, np.generic):
        return o.item()
    if isinstance(o, np.ndarray):
        return o.tolist()
    return str(o)


def load_model(path: str) -> Dict[str, Any]:
    with np.load(path, allow_pickle=False) as z:
        meta = json.loads(str(z["__meta__"]))
        for k in z.files:
            if k != "__meta__":
                meta[k] = z[k]
    return meta


_SAFE = re.compile(r"^[A-Za-z0-9_.\-]+$")


class ModelStore:
    def __init__(self, root: str):
        self.root = os.path.abspath(root)
        os.makedirs(self.root, exist_ok=True)

    def path_for(self, model_id: str) -> str:
        if not _SAFE.match(model_id):
            raise ValueError(f"invalid model id {model_id!r}")
        return os.path.join(self.root, f"{model_id}.npz")

    def save(self, model_id: str, model: Dict[str, Any]) -> str:
        return save_model(model, self.path_for(model_id))

    def resolve(self, model_path: Optional[str], model_id: Optional[str]) -> Optional[str]:
        """Only paths inside the store are served (no arbitrary file read)."""
        cands = []
        if model_id:
            try:
                cands.append(self.path_for(model_id))
            except ValueError:
                pass
        if model_path:
            p = os.path.abspath(model_path)
            if p.startswith(self.root + os.sep):
                cands.append(p)
        for c in cands:
            if os.path.isfile(c):
                return c
        return None


def predict(model: Dict[str, Any], X: np.ndarray) -> np.ndarray:
    """Predict raw feature rows on the CPU with the saved artefact."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    kind = model["kind"]
    classes = model.get("classes")
    if kind == "forest":
        from ..ops import forest_ops

        Xb = _bin_rows(model, X)
        fb = _forest_build(model)
        rows = np.arange(X.shape[0], dtype=np.int32)
        out = forest_ops.predict(fb, Xb, np.array([0, fb.n_trees]), np.array([0, X.shape[0]]), rows)
        return np.asarray(classes)[out] if (classes is not None and not fb.is_reg) else out
    if kind == "linear_logistic":
        z = X @ np.asarray(model["coef"]).T + np.asarray(model["intercept"])
        idx = (z[:, 0] > 0).astype(int) if z.shape[1] == 1 else z.argmax(1)
        return np.asarray(classes)[idx]
    if kind == "linear_regression":
        return X @ np.asarray(model["coef"]) + float(model["intercept"])
    if kind == "knn":
        from ..models.neighbors import knn_predict_numpy

        return knn_predict_numpy(model, X)
    if kind == "gbrt":
        from ..models.boosting import gbrt_predict_numpy

        return gbrt_predict_numpy(model, X)
    if kind == "svm":
        from ..models.svm import svm_predict_numpy

        return svm_predict_numpy(model, X)
    if kind == "pca":
        from ..models.transformers import pca_transform_numpy

        return pca_transform_numpy(model, X)   # a transformer's "prediction" is its projection
    raise ValueError(f"unknown model kind {kind!r}")


def _sigmoid(z: np.ndarray) -> np.ndarray:
    return 0.5 * (1.0 + np.tanh(0.5 * z))   # overflow-free logistic


def _softmax(z: np.ndarray) -> np.ndarray:
    z = z - z.max(1, keepdims=True)
    e = np.exp(z)
    return e / e.sum(1, keepdims=True)


_REGRESSOR_KINDS = ("linear_regression",)


class Predictor:
    """An estimator over a stored artefact (CPU; nothing from the file is executed).

    * ``predict(X)`` -- labels (classifiers, in the dataset's original label values) or values;
    * ``predict_proba(X)`` -- classifiers whose sklearn counterpart has it (forest, logistic,
      gradient boosting, k-NN); SVC has ``decision_function`` only (sklearn's default
      ``probability=False``);
    * ``score(X, y)`` -- accuracy (classifiers), R^2 (regressors), mean log-likelihood (PCA),
      the default ``score`` of the sklearn estimator and what a job reports as
      ``accuracy`` / ``r2_score`` / ``score``;
    * ``transform(X)`` -- PCA projection (whitened if the model was).
    """

    def __init__(self, model: Dict[str, Any]):
        self.model = model
        self.kind = str(model["kind"])
        self.model_type = str(model.get("model_type", self.kind))
        cl = model.get("classes")
        self.classes_ = None if cl is None else np.asarray(cl)
        if self.kind == "forest":
            self.is_classifier = not bool(model["is_reg"])
        elif self.kind == "svm":
            self.is_classifier = not bool(model["svr"])
        elif self.kind in ("pca",) + _REGRESSOR_KINDS:
            self.is_classifier = False
        else:
            self.is_classifier = self.classes_ is not None

    def __repr__(self) -> str:
        return f"Predictor({self.model_type}, kind={self.kind})"

    # ---- prediction --------------------------------------------------------------------
    def predict(self, X) -> np.ndarray:
        if self.kind == "pca":
            raise AttributeError("PCA has no predict; use transform / score")
        return predict(self.model, X)

    def decision_function(self, X) -> np.ndarray:
        X = np.ascontiguousarray(X, dtype=np.float32)
        if self.kind == "linear_logistic":
            z = X.astype(np.float64) @ np.asarray(self.model["coef"], dtype=np.float64).T + np.asarray(
                self.model["intercept"], dtype=np.float64)
            return z[:, 0] if z.shape[1] == 1 else z
        if self.kind == "gbrt" and self.is_classifier:
            from ..models.boosting import gbrt_raw_numpy

            raw = gbrt_raw_numpy(self.model, X)
            return raw[:, 0] if raw.shape[1] == 1 else raw
        if self.kind == "svm" and self.is_classifier and int(self.model["n_classes"]) == 2:
            from ..models.svm import _kernel_matrix
            import torch

            m = self.model["machines"][0]
            Xt = torch.from_numpy(X)
            sv = torch.from_numpy(np.asarray(m["sv"], dtype=np.float32).reshape(-1, X.shape[1]))
            K = _kernel_matrix(Xt, sv, int(self.model["kernel"]), float(self.model["gamma"]),
                               float(self.model["coef0"]), int(self.model["degree"]))
            dv = (K @ torch.from_numpy(np.asarray(m["coef"], dtype=np.float64)).to(K.dtype) - m["rho"]).numpy()
            return -dv   # sklearn's binary sign: positive -> classes_[1]
        raise AttributeError(f"{self.model_type} artefact has no decision_function")

    def predict_proba(self, X) -> np.ndarray:
        if not self.is_classifier:
            raise AttributeError(f"{self.model_type} is not a classifier")
        X = np.ascontiguousarray(X, dtype=np.float32)
        kind = self.kind
        if kind == "forest":
            from ..ops import forest_ops

            Xb = _bin_rows(self.model, X)
            fb = _forest_build(self.model)
            rows = np.arange(X.shape[0], dtype=np.int32)
            _, proba = forest_ops.predict(fb, Xb, np.array([0, fb.n_trees]), np.array([0, X.shape[0]]), rows,
                                          want_proba=True)
            return np.asarray(proba, dtype=np.float64)
        if kind == "linear_logistic":
            from ..models.linear import KIND_BINARY, KIND_OVR

            z = np.atleast_2d(self.decision_function(X).T).T
            link = int(self.model.get("link", KIND_BINARY))
            if z.shape[1] == 1:
                p1 = _sigmoid(z[:, 0])
                return np.stack([1.0 - p1, p1], 1)
            if link == KIND_OVR:   # sklearn one-vs-rest: normalised per-class sigmoids
                p = _sigmoid(z)
                return p / p.sum(1, keepdims=True)
            return _softmax(z)
        if kind == "gbrt":
            from ..models.boosting import LOSS_EXP, gbrt_raw_numpy

            raw = gbrt_raw_numpy(self.model, X)
            if raw.shape[1] == 1:
                p1 = _sigmoid(2.0 * raw[:, 0] if int(self.model["loss"]) == LOSS_EXP else raw[:, 0])
                return np.stack([1.0 - p1, p1], 1)
            return _softmax(raw)
        if kind == "knn":
            import torch

            from ..models.neighbors import finish_distance, knn_search_torch, vote

            m = self.model
            Xtr = torch.from_numpy(np.asarray(m["X"], dtype=np.float32))
            ytr = torch.from_numpy(np.asarray(m["y"]))
            Q = torch.from_numpy(X)
            n = Xtr.shape[0]
            metric, p, k = int(m["metric"]), float(m["p"]), int(m["n_neighbors"])
            acc, idx = knn_search_torch(torch.cat([Xtr, Q]), torch.arange(n, n + Q.shape[0]), torch.arange(n), k,
                                        metric, p)
            _, proba = vote(finish_distance(acc, metric, p), ytr[idx], k, m["weights"], int(m.get("n_classes", 1)),
                            True)
            return proba.numpy()
        raise AttributeError(f"{self.model_type} has no predict_proba (sklearn's default probability=False)")

    # ---- transformers ------------------------------------------------------------------
    def transform(self, X) -> np.ndarray:
        if self.kind != "pca":
            raise AttributeError(f"{self.model_type} has no transform")
        from ..models.transformers import pca_transform_numpy

        return pca_transform_numpy(self.model, X)

    def score_samples(self, X) -> np.ndarray:
        """PCA: per-row log-likelihood under the probabilistic PCA model (sklearn
        ``PCA.score_samples``): variance ``var_i`` (whitened: ``var_i (var_i - noise) + noise``)
        along each kept component, ``noise`` in the orthogonal complement."""
        if self.kind != "pca":
            raise AttributeError(f"{self.model_type} has no score_samples")
        m = self.model
        Xc = np.asarray(X, dtype=np.float64) - np.asarray(m["mean"], dtype=np.float64)
        comp = np.asarray(m["components"], dtype=np.float64)
        var = np.asarray(m["var"], dtype=np.float64)
        noise = float(m["noise_variance"])
        d, k = Xc.shape[1], comp.shape[0]
        if noise == 0.0 and k < d:
            return np.full(Xc.shape[0], -np.inf)
        lam = var * np.maximum(var - noise, 0.0) + noise if m.get("whiten") else np.where(var > noise, var, noise)
        Z = Xc @ comp.T
        resid = np.maximum((Xc * Xc).sum(1) - (Z * Z).sum(1), 0.0)
        quad = ((Z * Z) / lam).sum(1) + (resid / noise if k < d else 0.0)
        logdet = np.log(lam).sum() + ((d - k) * np.log(noise) if k < d else 0.0)
        return -0.5 * quad - 0.5 * (d * np.log(2 * np.pi) + logdet)

    def score(self, X, y=None) -> float:
        if self.kind == "pca":
            return float(np.mean(self.score_samples(X)))
        pred = self.predict(X)
        y = np.asarray(y)
        if self.is_classifier:
            return float(np.mean(pred == y))
        yv = y.astype(np.float64)
        ss_res = float(np.sum((yv - np.asarray(pred, dtype=np.float64)) ** 2))
        ss_tot = float(np.sum((yv - yv.mean()) ** 2))
        if ss_tot == 0.0:
            return 1.0 if ss_res == 0.0 else 0.0
        return 1.0 - ss_res / ss_tot


def _bin_rows(model: Dict[str, Any], X: np.ndarray) -> np.ndarray:
    from ..utils import native

    edges = np.ascontiguousarray(model["edges"], dtype=np.float32)
    Xb = np.empty(X.shape, dtype=np.uint8)
    native.cpu_lib().dml_cpu_bin(native.ptr(X), X.shape[0], X.shape[1], native.ptr(edges), native.ptr(Xb), X.shape[1])
    return Xb


def _forest_build(model: Dict[str, Any]):
    from ..ops import forest_ops

    return forest_ops.ForestBuild(np.ascontiguousarray(model["nodes"]), np.ascontiguousarray(model["vals"]),
                                  int(model["n_trees"]), int(model["vals"].shape[1]), bool(model["is_reg"]),
                                  int(model["n_classes"]))


def load_predictor(path: str) -> Predictor:
    """A downloaded ``.npz`` artefact as an estimator-like :class:`Predictor`."""
    return Predictor(load_model(path))
