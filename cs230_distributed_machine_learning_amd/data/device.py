"""Device-resident view of one dataset (the unit every fit of a job shares).

The reference worker reloads and re-splits the whole CSV for every task
(aws-prod/worker/worker.py:406-433, 302-303, 326).  Here a dataset is moved to the
device once (H2D, or an RCCL broadcast/all-gather across ranks — parallel/data.py),
its uint8 binned copy is built once on first tree use, and every CV/holdout split
is a row of a ``uint8 [S, n]`` role tensor (search/cv.py).  Fits only ever read these
resident buffers.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch

from ..search.cv import ROLE_TEST, ROLE_TRAIN


STREAM_CHUNK_ROWS = 1 << 20


class DeviceData:
    """``binned_only=True``: the float32 table never becomes resident.  It is streamed
    from host memory (numpy array or ``np.memmap``) in row chunks through two pinned
    buffers, with the H2D copy on a side stream overlapping the binning kernel of the
    previous chunk; only the uint8 bins stay in HBM (4x smaller: a 400 GB float32 table
    trains as 100 GB of bins).  The quantile edges come from the same 200k-row sample the
    resident path draws (ops/binning.py), so the bins -- and every tree -- are identical.
    Tree families run on the bins (``Family.binned_ok``); LinearRegression and PCA
    (``Family.streams_rows``) stream the host rows again in chunks (``stream_rows``)
    for their moments and test predictions; other families refuse such a table."""

    def __init__(self, X, y, classification: bool, device: torch.device | str = "cpu",
                 classes: Optional[np.ndarray] = None, name: str = "", binned_only: bool = False,
                 chunk_rows: int = STREAM_CHUNK_ROWS, _bins=None):
        self.device = torch.device(device)
        self.name = name
        self.binned_only = bool(binned_only)
        self._Xb = None
        self._edges = None
        self._X_host = None
        self._chunk_rows = int(chunk_rows)
        if self.binned_only:
            self.X = None
            Xh = X.cpu().numpy() if isinstance(X, torch.Tensor) else X
            self.n, self.d = Xh.shape
            self._X_host = Xh   # host (or memmap) rows: families with ``streams_rows`` read them in chunks
        elif isinstance(X, torch.Tensor):
            self.X = X.to(self.device, dtype=torch.float32).contiguous()
            self.n, self.d = self.X.shape
        else:
            self.X = torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32)).to(self.device)
            self.n, self.d = self.X.shape
        self.classification = bool(classification)
        self.y_is_numeric = True
        y_np = y.cpu().numpy() if isinstance(y, torch.Tensor) else np.asarray(y)
        self.y_host = y_np
        if self.classification:
            if classes is None:
                classes, y_enc = np.unique(y_np, return_inverse=True)
            else:
                lookup = {c: i for i, c in enumerate(classes.tolist())}
                y_enc = np.array([lookup[v] for v in y_np.tolist()], dtype=np.int64)
            self.classes = classes
            self.n_classes = len(classes)
            self.y_enc = y_enc.astype(np.int32)
            self.y_cls = torch.from_numpy(self.y_enc).to(self.device)
            self.y_reg = self.y_cls.float()
        else:
            self.classes = None
            self.n_classes = 1
            self.y_enc = None
            self.y_cls = None
            try:
                y_num = y_np.astype(np.float32)
                self.y_is_numeric = True
            except (ValueError, TypeError):
                # non-numeric target under a regressor / unsupervised estimator: keep codes so
                # unsupervised families (PCA) still run; regressors reject it (executor)
                y_num = np.unique(y_np.astype(str), return_inverse=True)[1].astype(np.float32)
                self.y_is_numeric = False
            self.y_reg = torch.from_numpy(y_num).to(self.device)
        if self.binned_only and _bins is not None:   # received bins (parallel/data.py broadcast_binned)
            self._Xb_full, self._edges, self._sample_max = _bins
            self._Xb = self._Xb_full[:, :self.d]
        elif self.binned_only:
            self._stream_bin(Xh, chunk_rows)
        self.roles = None
        self.split_names: List[str] = []
        self.test_rows: List[torch.Tensor] = []
        self.train_rows: List[torch.Tensor] = []
        self._split_key = None

    @property
    def is_gpu(self) -> bool:
        return self.device.type == "cuda"

    # ---- out-of-core float32 rows (binned-only tables) ---------------------------------
    def can_stream_rows(self) -> bool:
        return self.X is None and self._X_host is not None

    def stream_rows(self, chunk_rows: Optional[int] = None):
        """Yield (r0, r1, X[r0:r1] as float32 on the device) over a binned-only table's host
        rows: the float32 table never becomes resident, one chunk (and one pinned staging
        buffer) at a time.  The resident path keeps using ``self.X``."""
        if not self.can_stream_rows():
            raise ValueError("no host rows to stream (the table is resident or was received as bins)")
        Xh = self._X_host
        chunk = max(1, min(int(chunk_rows or self._chunk_rows), self.n))
        if not self.is_gpu:   # a fresh host array per chunk (the consumer may keep it)
            for r0 in range(0, self.n, chunk):
                r1 = min(self.n, r0 + chunk)
                yield r0, r1, torch.from_numpy(np.array(Xh[r0:r1], dtype=np.float32))
            return
        pin = torch.empty((chunk, self.d), dtype=torch.float32, pin_memory=True)
        for r0 in range(0, self.n, chunk):
            r1 = min(self.n, r0 + chunk)
            np.copyto(pin[:r1 - r0].numpy(), Xh[r0:r1], casting="same_kind")
            yield r0, r1, pin[:r1 - r0].to(self.device, non_blocking=False)

    def host_view(self) -> "DeviceData":
        """A CPU DeviceData over a binned-only table's host rows (same target, classes and
        name): the host solvers of families without a streamed or binned fit (SVC/SVR) train
        on it.  Made once per table; the caller sets its splits (executor.prepare_splits)."""
        if not self.can_stream_rows():
            raise ValueError("no host rows (the table is resident or was received as bins)")
        hv = getattr(self, "_host_view", None)
        if hv is None:
            hv = DeviceData(np.asarray(self._X_host, dtype=np.float32), self.y_host, self.classification, "cpu",
                            classes=self.classes, name=f"{self.name}@host")
            self._host_view = hv
        return hv

    # ---- binned copy (trees) -------------------------------------------------------
    def _stream_bin(self, Xh, chunk_rows: int) -> None:
        from ..ops import binning
        from ..utils import native

        n, d, dev = self.n, self.d, self.device
        sample = 200_000                                  # binning.quantile_edges' sample
        if n > sample:
            idx = np.sort(np.random.RandomState(0).choice(n, sample, replace=False))
            Xs = np.array(Xh[idx], dtype=np.float32, order="C")
        else:
            Xs = np.array(Xh, dtype=np.float32, order="C")
        Xs_t = torch.from_numpy(Xs).to(dev)
        self._edges = binning.quantile_edges(Xs_t)
        self._sample_max = Xs_t.max(0).values
        del Xs_t
        if not self.is_gpu:
            self._Xb = self._Xb_full = torch.empty((n, d), dtype=torch.uint8)
            for r0 in range(0, n, chunk_rows):
                r1 = min(n, r0 + chunk_rows)
                self._Xb[r0:r1] = binning.bin_matrix(torch.from_numpy(np.array(Xh[r0:r1], np.float32, order="C")),
                                                     self._edges)
            return
        ld = binning.row_pitch(d)
        buf = torch.zeros((n, ld), dtype=torch.uint8, device=dev)
        chunk = max(1, min(chunk_rows, n))
        pins = [torch.empty((chunk, d), dtype=torch.float32, pin_memory=True) for _ in range(2)]
        devb = [torch.empty((chunk, d), dtype=torch.float32, device=dev) for _ in range(2)]
        copy_stream = torch.cuda.Stream(dev)
        compute = torch.cuda.current_stream(dev)
        done = [None, None]
        lib = native.hip_lib()
        for i, r0 in enumerate(range(0, n, chunk)):
            b, m = i % 2, min(chunk, n - r0)
            if done[b] is not None:
                done[b].synchronize()                 # the chunk that last used buffer b is binned
            np.copyto(pins[b][:m].numpy(), Xh[r0:r0 + m], casting="same_kind")
            with torch.cuda.stream(copy_stream):
                devb[b][:m].copy_(pins[b][:m], non_blocking=True)
                copied = torch.cuda.Event()
                copied.record(copy_stream)
            compute.wait_event(copied)
            rc = lib.dml_bin(native.ptr(devb[b]), m, d, native.ptr(self._edges), native.ptr(buf[r0:r0 + m]), ld,
                             native.stream_handle(dev))
            if rc != 0:
                raise RuntimeError(f"dml_bin failed ({rc})")
            done[b] = torch.cuda.Event()
            done[b].record(compute)
        torch.cuda.synchronize(dev)
        self._Xb_full = buf
        self._Xb = buf[:, :d]

    @classmethod
    def from_bins(cls, Xb_full: torch.Tensor, d: int, edges: torch.Tensor, sample_max: torch.Tensor, y,
                  classification: bool, device, name: str = "") -> "DeviceData":
        """A binned-only table from bins built elsewhere (a broadcast from rank 0)."""
        n = Xb_full.shape[0]
        shape_only = np.lib.stride_tricks.as_strided(np.zeros(1, np.float32), (n, d), (0, 0))
        return cls(shape_only, y, classification, device, name=name, binned_only=True,
                   _bins=(Xb_full, edges, sample_max))

    def binned(self):
        if self._Xb is None:
            from ..ops import binning

            self._edges = binning.quantile_edges(self.X)
            self._Xb = binning.bin_matrix(self.X, self._edges)
        return self._Xb

    def binned_feature_major(self):
        """Feature-major copy of the bins, uint8 [d, n] (the forest builder's large tier
        gathers one feature of a dense sorted row set from it: coalesced)."""
        if getattr(self, "_XbT", None) is None:
            Xb = self.binned()
            self._XbT = Xb[:, :self.d].t().contiguous()
        return self._XbT

    def feature_major(self) -> torch.Tensor:
        """``X^T`` [d, n] contiguous (coalesced per-feature streaming in the KNN/SVM kernels)."""
        if self.X is None:
            raise ValueError("binned-only table: the float32 rows are not resident")
        if getattr(self, "_XT", None) is None:
            self._XT = self.X.t().contiguous()
        return self._XT

    def bin_values(self):
        """(values float32 [d, 256], exact uint8 [d]): the value each bin stands for, and
        whether EVERY row's value equals its bin's value (features with <= 256 distinct
        values).  Used to place split thresholds at sklearn's midpoints."""
        if getattr(self, "_binvals", None) is None and self.X is None:
            # binned-only: no rows to check exactness against -> thresholds stay at bin
            # boundaries (the midpoint refinement is skipped)
            E = self._edges
            finite = torch.isfinite(E)
            V = torch.full((self.d, 256), float("inf"), dtype=torch.float32, device=self.device)
            V[:, :255] = torch.where(finite, E, V[:, :255])
            V[torch.arange(self.d, device=self.device), finite.sum(1)] = self._sample_max
            self._binvals = (V.contiguous(), torch.zeros(self.d, dtype=torch.uint8, device=self.device))
        if getattr(self, "_binvals", None) is None:
            Xb = self.binned()
            E = self._edges
            finite = torch.isfinite(E)
            k = finite.sum(1)                                          # finite edges per feature
            V = torch.full((self.d, 256), float("inf"), dtype=torch.float32, device=self.device)
            V[:, :255] = torch.where(finite, E, V[:, :255])
            V[torch.arange(self.d, device=self.device), k] = self.X.max(0).values
            exact = torch.ones(self.d, dtype=torch.bool, device=self.device)
            step = max(1, (1 << 24) // max(1, self.d))
            for s0 in range(0, self.n, step):
                xb = Xb[s0:s0 + step].long()
                got = torch.gather(V, 1, xb.t()).t()
                exact &= (got == self.X[s0:s0 + step]).all(0)
            self._binvals = (V.contiguous(), exact.to(torch.uint8).contiguous())
        return self._binvals

    @property
    def edges(self):
        self.binned()
        return self._edges

    # ---- splits --------------------------------------------------------------------
    def set_splits(self, roles: np.ndarray, names: List[str], key=None) -> None:
        if key is not None and key == self._split_key:
            return
        roles = np.ascontiguousarray(roles, dtype=np.uint8)
        self.roles = torch.from_numpy(roles).to(self.device)
        self.split_names = list(names)
        self.test_rows = [torch.from_numpy(np.nonzero(r == ROLE_TEST)[0].astype(np.int32)).to(self.device) for r in roles]
        self.train_rows = [torch.from_numpy(np.nonzero(r == ROLE_TRAIN)[0].astype(np.int32)).to(self.device) for r in roles]
        self.train_counts = [int((r == ROLE_TRAIN).sum()) for r in roles]
        self._split_key = key

    def train_class_counts(self, split: int, C: int) -> torch.Tensor:
        """Per-class counts (float64 [C]) of a split's training rows."""
        yt = self.y_cls[self.train_rows[split].long()].long()
        return torch.bincount(yt, minlength=C).double()

    def test_targets(self, split: int) -> torch.Tensor:
        """Targets of a split's held-out rows, in the order predictions come back."""
        rows = self.test_rows[split].long()
        return (self.y_cls if self.classification else self.y_reg)[rows]

    def roles_np(self) -> np.ndarray:
        return self.roles.cpu().numpy()

    def sync(self):
        if self.is_gpu:
            torch.cuda.synchronize(self.device)
