"""Model artefacts: safe on-disk format + CPU/GPU prediction.

The reference pickles every fitted sklearn model into the worker's local
``./models/<subtask>_model.pkl`` (aws-prod/worker/worker.py:351-356) and the master
tries to ``send_file`` a path that only exists on the worker (D18).  Here artefacts
live in one shared model store as ``.npz`` (arrays + a JSON metadata string; loaded
with ``allow_pickle=False``, so downloading and loading a model executes nothing).

Kinds: ``forest`` (pool layout of ops/forest_ops.py + bin edges),
``linear_logistic``, ``linear_regression``, ``knn`` (training rows), ``gbrt`` (stage trees),
``svm`` (support vectors + dual coefficients per one-vs-one machine).
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
        from ..utils import native
        import torch

        lib = native.cpu_lib()
        edges = np.ascontiguousarray(model["edges"], dtype=np.float32)
        Xb = np.empty(X.shape, dtype=np.uint8)
        lib.dml_cpu_bin(native.ptr(X), X.shape[0], X.shape[1], native.ptr(edges), native.ptr(Xb), X.shape[1])
        fb = forest_ops.ForestBuild(np.ascontiguousarray(model["nodes"]), np.ascontiguousarray(model["vals"]),
                                    int(model["n_trees"]), int(model["vals"].shape[1]), bool(model["is_reg"]),
                                    int(model["n_classes"]))
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
    raise ValueError(f"unknown model kind {kind!r}")
