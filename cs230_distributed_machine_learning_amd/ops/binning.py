"""K1 — per-feature quantile edges and uint8 binning.

Edges are computed with torch on whichever device holds the table (sorting is exact,
positions are integer), so the CPU path and the GPU path produce identical edges and
therefore identical binned matrices.  Features with <= 256 distinct sampled values get
exact edges (all distinct values but the largest), so splits on low-cardinality
columns are exact like sklearn's; wider features get 255 sample quantiles.

The binning itself is the ``dml_bin`` HIP kernel on GPU and ``dml_cpu_bin`` (C++) on
CPU.  Reference context: the worker re-parses the whole CSV per task
(aws-prod/worker/worker.py:406-425); here a dataset is quantised once per device.
"""
from __future__ import annotations

import numpy as np
import torch

from ..utils import native

MAX_EDGES = 255


def quantile_edges(X: torch.Tensor, sample: int = 200_000, seed: int = 0) -> torch.Tensor:
    """float32 [d, 255] ascending edges, +inf padded, on X's device."""
    if X.dim() != 2:
        raise ValueError("X must be 2-D")
    n, d = X.shape
    if n > sample:
        idx = np.sort(np.random.RandomState(seed).choice(n, sample, replace=False))
        Xs = X[torch.from_numpy(idx).to(X.device)]
    else:
        Xs = X
    Xs = Xs.float()
    m = Xs.shape[0]
    S, _ = torch.sort(Xs, dim=0)
    # distinct-value count per feature
    diff = (S[1:] != S[:-1]).sum(dim=0) + 1 if m > 1 else torch.ones(d, dtype=torch.long, device=X.device)
    inf = torch.tensor(float("inf"), device=X.device)
    # quantile candidates at integer positions
    pos = torch.tensor([min(m - 1, ((i + 1) * m) // 256) for i in range(MAX_EDGES)], device=X.device)
    E = S[pos]  # [255, d]
    dup = torch.zeros_like(E, dtype=torch.bool)
    dup[1:] = E[1:] == E[:-1]
    # the largest sampled value never needs an edge (nothing in-sample lies above it)
    E = torch.where(dup | (E >= S[-1].unsqueeze(0)), inf, E)
    E, _ = torch.sort(E, dim=0)
    edges = E.t().contiguous()  # [d, 255]
    small = torch.nonzero(diff <= 256).flatten().tolist()
    for f in small:
        u = torch.unique(S[:, f])
        e = torch.full((MAX_EDGES,), float("inf"), device=X.device)
        if u.numel() > 1:
            e[: u.numel() - 1] = u[:-1]
        edges[f] = e
    return edges.float().contiguous()


def row_pitch(d: int) -> int:
    """Bytes per binned row on the GPU: whole rows per 128-byte cache line.

    The tree kernels gather a node's sampled features from each of its rows, so a row
    that straddles two lines costs two L2/MALL fetches; with d=100 unpadded, 77 % of
    rows straddle.  Rows of <= 128 bytes are padded to a power of two (so a line holds
    whole rows), wider rows to a multiple of 128.  ``DML_XB_PAD=0`` disables this."""
    import os

    if os.environ.get("DML_XB_PAD", "1") == "0":
        return d
    if d > 128:
        return (d + 127) // 128 * 128
    p = 4
    while p < d:
        p *= 2
    return p


def bin_matrix(X: torch.Tensor, edges: torch.Tensor) -> torch.Tensor:
    """uint8 [n, d] row-major bins of X (same device).  On the GPU the result is a
    [n, d] view of an [n, row_pitch(d)] buffer (consumers pass ``stride(0)``)."""
    X = X.float().contiguous()
    n, d = X.shape
    if X.is_cuda:
        ld = row_pitch(d)
        buf = torch.zeros((n, ld), dtype=torch.uint8, device=X.device)
        out = buf[:, :d]
        lib = native.hip_lib()
        rc = lib.dml_bin(native.ptr(X), n, d, native.ptr(edges), native.ptr(out), ld, native.stream_handle(X.device))
        if rc != 0:
            raise RuntimeError(f"dml_bin failed ({rc})")
    else:
        out = torch.empty((n, d), dtype=torch.uint8)
        lib = native.cpu_lib()
        lib.dml_cpu_bin(native.ptr(X), n, d, native.ptr(edges), native.ptr(out), d)
    return out
