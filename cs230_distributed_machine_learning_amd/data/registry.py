"""Dataset registry: ingest, lookup, load, metadata (reference C11 + the EFS layout).

Layout mirrors the reference's shared volume (aws-prod/master/config.py:11-18,
master/master.py:100-112): ``<root>/datasets/<name>/*.csv`` holds the raw file and
``<root>/datasets/<name>/preprocessed/*.csv`` the preprocessed one; preprocessing
YAMLs live in ``<root>/configs/<name>/``.  Loading prefers the preprocessed file and
falls back to the raw one (the reference only ever reads ``preprocessed/``,
worker.py:406).  ``feature_columns`` / ``target_column`` are honoured (D9); without
them the last column is the target like the reference (worker.py:428-429).

Sources (``download_data``): ``local`` (copy a file), ``sklearn`` (bundled toy
datasets: iris, wine, breast_cancer, diabetes, digits — available offline),
``synthetic`` (``"classification?n=1000&d=20&classes=2&seed=0"`` or ``regression?...``),
``huggingface`` / ``kaggle`` (attempted through their libraries when present; the
MI355X pool has no network so these report a clear error instead).
"""
from __future__ import annotations

import glob
import os
import shutil
import threading
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple
from urllib.parse import parse_qs

import numpy as np
import pandas as pd


@dataclass
class TabularDataset:
    name: str
    X: np.ndarray               # float32 [n, d]
    y: np.ndarray               # raw labels / targets
    feature_names: List[str]
    target_name: str
    path: Optional[str] = None
    metadata: Dict[str, Any] = field(default_factory=dict)

    @property
    def n(self) -> int:
        return int(self.X.shape[0])

    @property
    def d(self) -> int:
        return int(self.X.shape[1])


SKLEARN_SETS = ("iris", "wine", "breast_cancer", "diabetes", "digits", "california_housing")


class DatasetRegistry:
    def __init__(self, root: str):
        self.root = os.path.abspath(root)
        self.datasets_dir = os.path.join(self.root, "datasets")
        self.configs_dir = os.path.join(self.root, "configs")
        os.makedirs(self.datasets_dir, exist_ok=True)
        os.makedirs(self.configs_dir, exist_ok=True)
        self._cache: Dict[tuple, TabularDataset] = {}
        self._meta_cache: Dict[tuple, Dict[str, Any]] = {}
        self._lock = threading.Lock()

    # ---- paths -----------------------------------------------------------------------
    def dataset_dir(self, name: str) -> str:
        if not name or "/" in name or name.startswith(".") or "\\" in name:
            raise ValueError(f"invalid dataset name {name!r}")
        return os.path.join(self.datasets_dir, name)

    def find_file(self, name: str, preprocessed_first: bool = True) -> Optional[str]:
        d = self.dataset_dir(name)
        pats = ["*.csv", "*.parquet", "*.npz"]
        cands: List[str] = []
        if preprocessed_first:
            for p in pats:
                cands += sorted(glob.glob(os.path.join(d, "preprocessed", p)))
        for p in pats:
            cands += sorted(glob.glob(os.path.join(d, p)))
        return cands[0] if cands else None

    def raw_file(self, name: str) -> Optional[str]:
        return self.find_file(name, preprocessed_first=False)

    # ---- ingest ----------------------------------------------------------------------
    def download(self, url: str, source_type: str, name: str) -> Tuple[bool, str]:
        try:
            dest = self.dataset_dir(name)
            os.makedirs(dest, exist_ok=True)
            st = (source_type or "").lower()
            if st == "local":
                if not os.path.isfile(url):
                    return False, f"Local file not found at path: {url}"
                shutil.copy(url, dest)
            elif st == "sklearn":
                self._write_frame(self._sklearn_frame(url), os.path.join(dest, f"{name}.csv"))
            elif st == "synthetic":
                X, y, cols = synthetic_table(url)
                if X.shape[0] * X.shape[1] > 20_000_000:
                    np.savez(os.path.join(dest, f"{name}.npz"), X=X, y=y, columns=np.array(cols))
                else:
                    df = pd.DataFrame(X, columns=cols[:-1])
                    df[cols[-1]] = y
                    self._write_frame(df, os.path.join(dest, f"{name}.csv"))
            elif st == "huggingface":
                try:
                    from datasets import load_dataset  # noqa: F401
                except ImportError:
                    return False, "huggingface `datasets` is not installed"
                from datasets import load_dataset

                ds = load_dataset(url)
                split = ds[list(ds.keys())[0]]
                self._write_frame(split.to_pandas(), os.path.join(dest, f"{name}.csv"))
            elif st == "kaggle":
                try:
                    import kaggle  # noqa: F401
                except Exception as e:  # kaggle raises on import without credentials
                    return False, f"kaggle source unavailable: {e}"
                kaggle.api.dataset_download_files(url, path=dest, unzip=True)
            else:
                return False, f"Invalid source type: {source_type}"
            self.invalidate(name)
            return True, f"Dataset downloaded successfully to {dest}"
        except Exception as e:  # surfaced as 500 like the reference
            return False, f"{type(e).__name__}: {e}"

    @staticmethod
    def _write_frame(df: pd.DataFrame, path: str) -> None:
        df.to_csv(path, index=False)

    @staticmethod
    def _sklearn_frame(which: str) -> pd.DataFrame:
        import sklearn.datasets as skd

        which = which.lower()
        if which not in SKLEARN_SETS:
            raise ValueError(f"unknown sklearn dataset {which!r}; choose from {SKLEARN_SETS}")
        if which == "california_housing":
            b = skd.fetch_california_housing(as_frame=True)
        else:
            b = getattr(skd, f"load_{which}")(as_frame=True)
        df = b.frame.copy()
        if which == "iris":
            df.columns = ["sepal_length", "sepal_width", "petal_length", "petal_width", "species"]
            df["species"] = np.array(b.target_names)[b.target]
        return df

    def save_preprocessed(self, name: str, df: pd.DataFrame) -> str:
        d = os.path.join(self.dataset_dir(name), "preprocessed")
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, f"{name}_preprocessed.csv")
        df.to_csv(path, index=False)
        self.invalidate(name)
        return path

    def invalidate(self, name: str) -> None:
        with self._lock:
            for k in [k for k in self._cache if k[0] == name]:
                del self._cache[k]

    # ---- load --------------------------------------------------------------------------
    def load(self, name: str, feature_columns: Optional[List[str]] = None,
             target_column: Optional[str] = None) -> TabularDataset:
        path = self.find_file(name)
        if path is None:
            raise FileNotFoundError(f"Dataset {name} not found, Please Use download_data function")
        key = (name, path, os.path.getmtime(path), tuple(feature_columns or ()), target_column or "")
        with self._lock:
            if key in self._cache:
                return self._cache[key]
        ds = load_table(path, name, feature_columns, target_column)
        with self._lock:
            self._cache[key] = ds
        return ds

    def metadata(self, name: str) -> Dict[str, Any]:
        """{n_rows, n_cols, size_mb}, cached per (file, mtime): the cluster dispatcher asks at
        every job admission, and counting a large CSV's rows would stall it for seconds."""
        path = self.find_file(name)
        if path is None:
            return {}
        key = ("__meta__", path, os.path.getmtime(path))
        with self._lock:
            hit = self._meta_cache.get(key)
        if hit is None:
            hit = file_metadata(path)
            with self._lock:
                self._meta_cache[key] = hit
        return dict(hit)


def file_metadata(path: str) -> Dict[str, Any]:
    """{n_rows, n_cols, size_mb} — reference dataset_util.py:119-137."""
    size_mb = round(os.path.getsize(path) / (1024 * 1024), 2)
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            n, d = z["X"].shape
        return {"n_rows": int(n), "n_cols": int(d) + 1, "size_mb": size_mb}
    if path.endswith(".parquet"):
        df = pd.read_parquet(path)
        return {"n_rows": int(len(df)), "n_cols": int(df.shape[1]), "size_mb": size_mb}
    with open(path, "r", encoding="utf-8", newline="") as f:
        header = f.readline()
        rows = sum(1 for _ in f)
    return {"n_rows": rows, "n_cols": len(header.split(",")), "size_mb": size_mb}


def load_table(path: str, name: str, feature_columns=None, target_column=None) -> TabularDataset:
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            X, y = z["X"].astype(np.float32), z["y"]
            cols = [str(c) for c in z["columns"]] if "columns" in z else [f"x{i}" for i in range(X.shape[1])] + ["y"]
        return TabularDataset(name, np.ascontiguousarray(X), y, cols[:-1], cols[-1], path, file_metadata(path))
    df = pd.read_parquet(path) if path.endswith(".parquet") else pd.read_csv(path)
    if target_column and target_column in df.columns:
        tcol = target_column
    else:
        tcol = df.columns[-1]
    if feature_columns:
        missing = [c for c in feature_columns if c not in df.columns]
        if missing:
            raise ValueError(f"feature_columns not in dataset: {missing}")
        fcols = list(feature_columns)
    else:
        fcols = [c for c in df.columns if c != tcol]
    Xdf = df[fcols]
    # non-numeric features: stable category codes (documented deviation; preprocess first)
    for c in Xdf.columns:
        if not pd.api.types.is_numeric_dtype(Xdf[c]):
            Xdf = Xdf.assign(**{c: pd.factorize(Xdf[c].astype(str), sort=True)[0]})
    X = Xdf.to_numpy(dtype=np.float32, na_value=np.nan)
    y = df[tcol].to_numpy()
    return TabularDataset(name, np.ascontiguousarray(X), y, [str(c) for c in fcols], str(tcol), path,
                          file_metadata(path))


def synthetic_table(spec: str, seed_default: int = 0):
    """``classification?n=..&d=..&classes=..&informative=..&seed=..`` or ``regression?...``;
    ``&gen=blocks`` uses the block generator of data/synthetic.py (n a multiple of 15625)."""
    kind, _, q = spec.partition("?")
    args = {k: v[0] for k, v in parse_qs(q).items()}
    n = int(args.get("n", 1000))
    d = int(args.get("d", 20))
    seed = int(args.get("seed", seed_default))
    if args.get("gen") == "blocks":
        # the block generator of data/synthetic.py (what bench.py makes on the device):
        # same weights and noise model, so bench --e2e fits the bench's table shape AND
        # difficulty (tree sizes follow the label noise)
        from . import synthetic as _syn

        reg = not kind.startswith("class")
        Xt, yt = _syn.make_table(n, d, informative=int(args.get("informative", min(d, 10))),
                                 n_classes=int(args.get("classes", 2)), noise=float(args.get("noise", 1.0)), seed=seed,
                                 device="cpu", regression=reg)
        X, y = Xt.numpy(), (yt.numpy() if reg else yt.numpy().astype(np.int64))
    else:
        X, y = synthetic_arrays(kind, n, d, int(args.get("classes", 2)), int(args.get("informative", min(d, 10))),
                                seed, float(args.get("noise", 0.5)))
    cols = [f"x{i}" for i in range(d)] + ["target"]
    return X, y, cols


def synthetic_arrays(kind: str, n: int, d: int, classes: int = 2, informative: int = 10, seed: int = 0,
                     noise: float = 0.5):
    """Deterministic synthetic tabular data (numpy; the device version is data/synthetic.py)."""
    rng = np.random.RandomState(seed)
    X = rng.standard_normal((n, d)).astype(np.float32)
    informative = max(1, min(informative, d))
    W = rng.standard_normal((informative, max(1, classes if kind.startswith("class") else 1))).astype(np.float32)
    logits = X[:, :informative] @ W + noise * rng.standard_normal((n, W.shape[1])).astype(np.float32)
    if kind.startswith("class"):
        y = (logits[:, 0] > 0).astype(np.int64) if classes == 2 else np.argmax(logits, 1).astype(np.int64)
    else:
        y = logits[:, 0].astype(np.float32)
    return X, y
