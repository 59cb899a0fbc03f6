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


class DeviceData:
    def __init__(self, X, y, classification: bool, device: torch.device | str = "cpu",
                 classes: Optional[np.ndarray] = None, name: str = ""):
        self.device = torch.device(device)
        self.name = name
        if isinstance(X, torch.Tensor):
            self.X = X.to(self.device, dtype=torch.float32).contiguous()
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
        self._Xb = None
        self._edges = None
        self.roles = None
        self.split_names: List[str] = []
        self.test_rows: List[torch.Tensor] = []
        self.train_rows: List[torch.Tensor] = []
        self._split_key = None

    @property
    def is_gpu(self) -> bool:
        return self.device.type == "cuda"

    # ---- binned copy (trees) -------------------------------------------------------
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
        if getattr(self, "_XT", None) is None:
            self._XT = self.X.t().contiguous()
        return self._XT

    def bin_values(self):
        """(values float32 [d, 256], exact uint8 [d]): the value each bin stands for, and
        whether EVERY row's value equals its bin's value (features with <= 256 distinct
        values).  Used to place split thresholds at sklearn's midpoints."""
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
