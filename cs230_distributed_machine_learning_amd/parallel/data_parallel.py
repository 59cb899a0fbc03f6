"""Row-sharded data-parallel fits: one job's fits run on ALL ranks at once.

The reference has only task parallelism (one candidate per worker; every
worker re-reads the full CSV, aws-prod/worker/worker.py:406-425).  Task parallelism is
this framework's default too (parallel/runner.py), but it needs a full copy of the table
per GPU and at least one slice per rank.  Data-parallel mode covers the other two
cases — a table larger than one GPU wants to hold, or fewer fits than ranks:

* ``scatter_table``: rank 0 parses the table once; every rank receives only its
  contiguous row block ``[r0, r1)`` (chunked RCCL point-to-point sends; rank 0's device
  holds its own block plus one chunk).  Labels are tiny
  and are broadcast whole, so every rank builds the SAME global CV/holdout split roles.
* ``RowShard``: a ``DeviceData`` over the local rows whose split bookkeeping is global:
  local ``roles``/``train_rows``/``test_rows`` index the shard, ``train_counts`` and
  class statistics are the global ones (objective scale ``1/n_train`` is global).
* Families that declare ``data_parallel = True`` reduce their sufficient statistics
  through ``RowShard.all_reduce``: LogisticRegression sums per-rank loss and gradient
  ``X_r^T R_r`` (one all-reduce of the [d+1, M] gradient per objective evaluation,
  every rank then takes the identical batched L-BFGS step); LinearRegression sums the
  normal equations ``X^T X``, ``X^T y``.
* Held-out predictions stay on their rank; ``gather_outputs`` all-gathers them (ranks'
  test rows concatenate in global row order) so scoring sees exactly the single-GPU
  prediction vector.

Over xGMI the per-evaluation all-reduce is (d+1) x M x 4 bytes (512 fits x 1001 x 4 =
2 MB): a few microseconds of link time against a GEMM over the shard's rows.
"""
from __future__ import annotations

import json
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..data.device import DeviceData
from ..search.cv import ROLE_TEST, ROLE_TRAIN
from . import dist


SCATTER_CHUNK_BYTES = 256 << 20


def shard_bounds(n: int, world: int, rank: int):
    """Contiguous row block of ``rank``: sizes differ by at most one row."""
    base, rem = divmod(n, world)
    r0 = rank * base + min(rank, rem)
    return r0, r0 + base + (1 if rank < rem else 0)


def _guarded(fn):
    """Run a collective of a row-sharded epoch; any failure (timeout on a dead or hung peer,
    communicator abort) becomes ``dist.CollectiveError``, which aborts the epoch."""
    try:
        return fn()
    except dist.CollectiveError:
        raise
    except Exception as e:
        raise dist.CollectiveError(f"row-shard collective failed: {type(e).__name__}: {e}") from e


def scatter_table(X: Optional[np.ndarray], y: Optional[np.ndarray], device: torch.device, group=None):
    """Rank 0 passes host arrays; every rank returns (X_shard_dev, y_global_host, r0).

    X moves by chunked point-to-point sends from rank 0 (each rank receives only its
    rows; rank 0 holds its own block plus one chunk); y (n values) is broadcast to
    every rank.  ``group``: the data-parallel communicator (dist.dp_group; its ranks are
    the global ranks)."""
    inf = dist.info()
    if not inf.is_dist:
        return torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32)).to(device), np.asarray(y), 0
    return _guarded(lambda: _scatter(X, y, device, group))


def _scatter(X, y, device, group):
    import datetime

    inf = dist.info()
    st = dist.store()
    key = "dataset/dp_meta"
    if inf.rank == 0:
        y = np.asarray(y)
        if y.dtype.kind in "OUS":
            classes, codes = np.unique(y.astype(str), return_inverse=True)
            meta = {"n": int(X.shape[0]), "d": int(X.shape[1]), "y": "codes", "classes": classes.tolist()}
            y_num = codes.astype(np.float64)
        else:
            meta = {"n": int(X.shape[0]), "d": int(X.shape[1]), "y": str(y.dtype)}
            y_num = y.astype(np.float64)
        st.set(key, json.dumps(meta))
    else:
        st.wait([key], datetime.timedelta(seconds=dist.dp_timeout_s() if group is not None else 1800.0))
        meta = json.loads(st.get(key))
    n, d, world = meta["n"], meta["d"], inf.world
    r0, r1 = shard_bounds(n, world, inf.rank)
    recv = torch.empty((r1 - r0, d), dtype=torch.float32, device=device)
    # rank 0 keeps only its own block resident: every other rank's rows leave in
    # row chunks of <= SCATTER_CHUNK_BYTES, one point-to-point send at a time, so rank 0's
    # device never holds more than its block plus one chunk (a table larger than one GPU
    # wants to hold is exactly what this mode is for)
    ch = max(1, SCATTER_CHUNK_BYTES // max(1, 4 * d))
    if inf.rank == 0:
        Xt = torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32))
        recv.copy_(Xt[r0:r1])
        for k in range(1, world):
            a, b = shard_bounds(n, world, k)
            for c0 in range(a, b, ch):
                c1 = min(b, c0 + ch)
                torch.distributed.send(Xt[c0:c1].to(device), dst=k, group=group)
    else:
        for c0 in range(r0, r1, ch):
            c1 = min(r1, c0 + ch)
            torch.distributed.recv(recv[c0 - r0:c1 - r0], src=0, group=group)
    yd = torch.from_numpy(y_num).to(device) if inf.rank == 0 else torch.empty((n,), dtype=torch.float64, device=device)
    dist.broadcast(yd, 0, group=group)
    dist.barrier(group=group)
    if inf.rank == 0:
        st.delete_key(key)
        return recv, y, r0
    y_host = yd.cpu().numpy()
    if meta["y"] == "codes":
        y_host = np.asarray(meta["classes"], dtype=object)[y_host.astype(np.int64)]
    else:
        y_host = y_host.astype(np.dtype(meta["y"]))
    return recv, y_host, r0


class RowShard(DeviceData):
    """This rank's rows ``[r0, r0 + n)`` of a global table, with global split semantics."""

    is_row_shard = True

    def __init__(self, X_shard, y_global: np.ndarray, r0: int, classification: bool, device, name: str = "",
                 group=None):
        y_global = np.asarray(y_global)
        n_loc = int(X_shard.shape[0])
        classes = np.unique(y_global) if classification else None
        super().__init__(X_shard, y_global[r0:r0 + n_loc], classification, device, classes=classes, name=name)
        self.r0, self.n_global = int(r0), int(len(y_global))
        self.y_host = y_global            # split construction (stratified folds) sees the global labels
        self.group = group
        if self.classification:   # classes come sorted from np.unique: codes by binary search
            codes = np.searchsorted(classes, y_global).astype(np.int32)
            self._y_glob = torch.from_numpy(codes).to(self.device)
        else:
            self._y_glob = torch.from_numpy(np.asarray(y_global, dtype=np.float32)).to(self.device)
        self._test_glob: List[torch.Tensor] = []
        self._test_counts: List[np.ndarray] = []

    # ---- collectives ------------------------------------------------------------------
    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """In-place sum / min / max over ranks (RCCL on GPU, gloo on CPU); identical
        result on every rank."""
        if dist.info().is_dist:
            ro = {"sum": torch.distributed.ReduceOp.SUM, "min": torch.distributed.ReduceOp.MIN,
                  "max": torch.distributed.ReduceOp.MAX}[op]
            _guarded(lambda: torch.distributed.all_reduce(t, op=ro, group=self.group))
        return t

    # reduce-scatter / all-gather over equal row blocks (row-sharded forests: each rank
    # owns 1/N of a level's node histograms, evaluates them, and shares the decisions)
    @property
    def world(self) -> int:
        return dist.info().world if dist.info().is_dist else 1

    @property
    def rank(self) -> int:
        return dist.info().rank if dist.info().is_dist else 0

    def reduce_scatter_rows(self, t: torch.Tensor) -> torch.Tensor:
        """Sum over ranks of ``t`` [world * q, ...]; this rank gets rows [rank*q, rank*q+q)."""
        w = self.world
        if w == 1:
            return t
        q = t.shape[0] // w
        if dist.info().backend == "nccl":
            out = torch.empty((q,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            _guarded(lambda: torch.distributed.reduce_scatter_tensor(out, t.contiguous(), group=self.group))
            return out
        _guarded(lambda: torch.distributed.all_reduce(t, group=self.group))    # gloo: no reduce-scatter
        return t[self.rank * q:(self.rank + 1) * q]

    def all_gather_equal(self, t: torch.Tensor) -> torch.Tensor:
        """Rank-ordered concatenation of every rank's equal-size ``t``."""
        w = self.world
        if w == 1:
            return t
        t = t.contiguous()
        if dist.info().backend == "nccl":
            out = torch.empty((w * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            _guarded(lambda: torch.distributed.all_gather_into_tensor(out, t, group=self.group))
            return out
        parts = [torch.empty_like(t) for _ in range(w)]
        _guarded(lambda: torch.distributed.all_gather(parts, t, group=self.group))
        return torch.cat(parts)

    def _world_bounds(self):
        world = dist.info().world if dist.info().is_dist else 1
        return [shard_bounds(self.n_global, world, k) for k in range(world)] if world > 1 else [(0, self.n_global)]

    # ---- binned copy (row-sharded forests) --------------------------------------------
    def binned(self):
        """Bins of the local rows with the GLOBAL quantile edges: the 200k-row edge sample
        of ops/binning.py is drawn over global row ids, every rank contributes its sampled
        rows and one all-gather assembles the sample in global row order -- so the edges,
        and every tree, equal the single-GPU ones."""
        if self._Xb is None:
            from ..ops import binning

            sample = 200_000
            if self.n_global > sample:
                idx = np.sort(np.random.RandomState(0).choice(self.n_global, sample, replace=False))
            else:
                idx = np.arange(self.n_global)
            loc = idx[(idx >= self.r0) & (idx < self.r0 + self.n)] - self.r0
            Xs = self.X[torch.from_numpy(loc).to(self.device)]
            counts = np.array([int(((idx >= a) & (idx < b)).sum()) for a, b in self._world_bounds()], dtype=np.int64)
            Xs = self._gather_rows(Xs, counts)
            self._edges = binning.quantile_edges(Xs)
            self._Xb = binning.bin_matrix(self.X, self._edges)
        return self._Xb

    def bin_values(self):
        """``DeviceData.bin_values`` over the global table: the top bin's value is the
        global column max, and a feature is exactly binned only if it is on every rank."""
        if getattr(self, "_binvals", None) is None:
            Xb = self.binned()
            E = self._edges
            finite = torch.isfinite(E)
            k = finite.sum(1)
            V = torch.full((self.d, 256), float("inf"), dtype=torch.float32, device=self.device)
            V[:, :255] = torch.where(finite, E, V[:, :255])
            mx = self.X.max(0).values if self.n else torch.full((self.d,), float("-inf"), device=self.device)
            V[torch.arange(self.d, device=self.device), k] = self.all_reduce(mx.contiguous(), "max")
            exact = torch.ones(self.d, dtype=torch.bool, device=self.device)
            step = max(1, (1 << 24) // max(1, self.d))
            for s0 in range(0, self.n, step):
                got = torch.gather(V, 1, Xb[s0:s0 + step].long().t()).t()
                exact &= (got == self.X[s0:s0 + step]).all(0)
            ex = self.all_reduce(exact.to(torch.int32), "min")
            self._binvals = (V.contiguous(), ex.to(torch.uint8).contiguous())
        return self._binvals

    def _gather_rows(self, t: torch.Tensor, counts: np.ndarray) -> torch.Tensor:
        if not dist.info().is_dist:
            return t
        m = int(counts.max()) if len(counts) else 0
        pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[:t.shape[0]] = t
        parts = [torch.empty_like(pad) for _ in counts]
        _guarded(lambda: torch.distributed.all_gather(parts, pad, group=self.group))
        return torch.cat([p[:int(c)] for p, c in zip(parts, counts)])

    # ---- splits -----------------------------------------------------------------------
    def set_splits(self, roles: np.ndarray, names: List[str], key=None) -> None:
        if key is not None and key == self._split_key:
            return
        roles = np.ascontiguousarray(roles, dtype=np.uint8)
        n_loc = self.n
        world = dist.info().world if dist.info().is_dist else 1
        loc = np.ascontiguousarray(roles[:, self.r0:self.r0 + n_loc])
        super().set_splits(loc, names, key=None)
        self._split_key = key
        self.train_counts = [int((r == ROLE_TRAIN).sum()) for r in roles]          # global
        self._test_glob = [torch.from_numpy(np.nonzero(r == ROLE_TEST)[0].astype(np.int64)).to(self.device)
                           for r in roles]
        bounds = self._world_bounds()
        self._test_counts = [np.array([int((r[a:b] == ROLE_TEST).sum()) for a, b in bounds], dtype=np.int64)
                             for r in roles]
        if world > 1 and bounds[dist.info().rank] != (self.r0, self.r0 + n_loc):
            raise ValueError("RowShard rows do not match shard_bounds for this rank")

    def train_class_counts(self, split: int, C: int) -> torch.Tensor:
        """Global per-class counts of a split's training rows."""
        yt = self.y_cls[self.train_rows[split].long()].long()
        return self.all_reduce(torch.bincount(yt, minlength=C).double())

    def test_targets(self, split: int) -> torch.Tensor:
        return self._y_glob[self._test_glob[split]]

    def gather_outputs(self, tasks: Sequence, outputs: Dict[int, object]) -> None:
        """Replace every output's local test predictions by the global ones (rank order =
        global row order).  Every rank holds the same tasks, so the collectives match."""
        for t in sorted(tasks, key=lambda t: t.task_id):
            o = outputs.get(t.task_id)
            if o is None or o.pred is None:   # self-scored families (PCA) reduce their own score
                continue
            cnt = self._test_counts[t.split]
            o.pred = self._gather_rows(o.pred, cnt)
            if o.proba is not None:
                o.proba = self._gather_rows(o.proba, cnt)
            if getattr(o, "decision", None) is not None:
                o.decision = self._gather_rows(o.decision, cnt)
