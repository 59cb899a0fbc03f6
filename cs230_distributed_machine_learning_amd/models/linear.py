"""LogisticRegression and LinearRegression families — every fit of a job solved at once.

Reference: both are whitelisted estimators fitted one (candidate, fold) at a time by
sklearn on CPU (aws-prod/worker/worker.py:39,46 whitelist; :315, :326/:341 fits).

LogisticRegression
    Each fit (candidate x split) owns a block of columns of ONE weight matrix
    ``W [d+1, M]`` (last row = intercept).  Per objective evaluation the whole batch
    does: ``Z = X @ W`` (library GEMM) -> fused HIP link/loss/residual kernel
    (``dml_lr_link_grad``, csrc/kernels/linear.hip) -> ``G = X^T R`` (library GEMM).
    A batched L-BFGS (per-fit histories, per-fit Armijo steps, per-fit stopping on
    ``max|grad| <= tol`` or ``max_iter``) minimises every fit's objective
    ``mean(loss) + ||w||^2 / (2 C n)`` — the same optimum sklearn's lbfgs /
    newton-cg / sag(a) / liblinear reach (liblinear: one-vs-rest, intercept
    penalised via ``intercept_scaling``).  Binary problems use one sigmoid column,
    multiclass the multinomial softmax (or OvR columns for liblinear / multi_class='ovr').
LinearRegression
    Normal equations per split (shared by every candidate on that split), solved by
    pseudo-inverse (min-norm like sklearn's lstsq).  On the GPU every split's moments
    come from one fused pass over X (``dml_split_moments``: f64 MFMA tiles, split
    masks from the role rows, shifted by the column means for an accurate centring).
"""
from __future__ import annotations

import ctypes
import math
import os
import time
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from ..utils import native, trace
from .base import Family, FitOutput, FitTask, ParamError, as_bool, as_float, as_int, register, seed_of

KIND_BINARY, KIND_SOFTMAX, KIND_OVR = 0, 1, 2

_LR_DEFAULTS = {
    "penalty": "l2", "dual": False, "tol": 1e-4, "C": 1.0, "fit_intercept": True, "intercept_scaling": 1.0,
    "class_weight": None, "random_state": None, "solver": "lbfgs", "max_iter": 100, "multi_class": "deprecated",
    "verbose": 0, "warm_start": False, "n_jobs": None, "l1_ratio": None,
}
_SOLVERS = ("lbfgs", "liblinear", "newton-cg", "newton-cholesky", "sag", "saga")


def link_grad_torch(Z: torch.Tensor, y: torch.Tensor, roles: torch.Tensor, col0, K, kind, split, scale, cw=None):
    """Reference (CPU) implementation of the fused kernel: returns (R, loss[F]).

    Vectorised over fits sharing a (link kind, width) so a batch costs a handful of
    tensor ops regardless of how many candidates x folds it holds.
    """
    n, M = Z.shape
    F = len(col0)
    R = torch.zeros_like(Z)
    loss = torch.zeros(F, dtype=torch.float64, device=Z.device)
    yl = y.long()
    groups: Dict[tuple, List[int]] = {}
    for f in range(F):
        groups.setdefault((int(kind[f]), int(K[f])), []).append(f)
    for (kd, k), fits in groups.items():
        fi = torch.tensor(fits, dtype=torch.long, device=Z.device)
        cols = (torch.tensor([int(col0[f]) for f in fits], device=Z.device).view(-1, 1)
                + torch.arange(k, device=Z.device).view(1, -1))                      # [G, k]
        z = Z[:, cols.flatten()].view(n, len(fits), k)                                 # [n, G, k]
        m = (roles[torch.tensor([int(split[f]) for f in fits], device=Z.device)] == 1).t().to(Z.dtype)  # [n, G]
        s = torch.tensor([float(scale[f]) for f in fits], dtype=Z.dtype, device=Z.device).view(1, -1)
        if kd == KIND_SOFTMAX:
            lse = torch.logsumexp(z, dim=2, keepdim=True)
            onehot = torch.nn.functional.one_hot(yl, k).to(Z.dtype).unsqueeze(1)
            r = torch.exp(z - lse) - onehot
            l = lse.squeeze(2) - z.gather(2, yl.view(-1, 1, 1).expand(n, len(fits), 1)).squeeze(2)
        else:
            if kd == KIND_BINARY:
                tgt = (yl == 1).to(Z.dtype).view(n, 1, 1).expand(n, len(fits), 1)
            else:
                tgt = torch.nn.functional.one_hot(yl, k).to(Z.dtype).unsqueeze(1).expand(n, len(fits), k)
            r = torch.sigmoid(z) - tgt
            l = torch.nn.functional.softplus(torch.where(tgt > 0.5, -z, z)).sum(2)
        if cw is not None:   # per-row class weight of each fit (sample weights by class)
            m = m * cw[fi][:, yl].t().to(Z.dtype)
        r = r * (m * s).unsqueeze(2)
        R[:, cols.flatten()] = r.reshape(n, -1)
        loss[fi] = (l.double() * m.double()).sum(0) * s.squeeze(0).double()
    return R, loss


def class_weight_vector(data, split: int, cw):
    """sklearn ``compute_class_weight`` on the split's training rows (None: unweighted)."""
    if cw is None:
        return None
    C = data.n_classes
    w = torch.ones(C, dtype=torch.float64, device=data.device)
    if cw == "balanced":
        cnt = data.train_class_counts(split, C)      # global counts under a RowShard
        return torch.where(cnt > 0, cnt.sum() / (C * cnt.clamp_min(1)), w)
    lookup = {str(c): i for i, c in enumerate(np.asarray(data.classes).tolist())}
    for k, v in cw.items():
        if str(k) in lookup:
            w[lookup[str(k)]] = float(v)
    return w


_TILE = 128   # output tile of csrc/kernels/lr_mfma.hip (dml_lr_mfma_tile): a fit's columns never straddle one
_ROW_TILE = 256   # v3 kernels' row tile (dml_lr_v3_row_tile): X rows and R^T rows (= padded columns)


def lr_v3(lib, M: int) -> bool:
    """The 3-stage 256 x 128 MFMA kernels (k_lr_fwd3 / k_lr_grad3, one workgroup per CU) for
    batches of more than 256 columns; smaller batches keep the 128 x 128 two-workgroup kernels
    (a 256-row gradient tile would be mostly padding).  DML_LR_V3=0 forces the older kernels."""
    return (M > 256 and os.environ.get("DML_LR_V3", "1") != "0"
            and getattr(lib, "dml_lr_mfma_fwd3", None) is not None)


def _dp_sum(data, t: torch.Tensor) -> torch.Tensor:
    """Sum over the ranks of a row-sharded fit (parallel/data_parallel.py); identity otherwise."""
    if getattr(data, "is_row_shard", False):
        t = t.contiguous()
        data.all_reduce(t)
    return t


def _roundup(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def mfma_enabled(data) -> bool:
    """The matrix-core objective runs for every device batch unless DML_LR_MFMA=0."""
    return data.is_gpu and os.environ.get("DML_LR_MFMA", "1") != "0"


def fold_grouped_perm(roles: torch.Tensor) -> torch.Tensor:
    """Row order that groups rows with the same role in every split: a stable sort by the
    role tuple (split 0 most significant).  For k-fold CV every fold's rows become ONE
    contiguous block, so each split's non-training rows fill whole 256-row tiles that its
    fits' objective can skip (they only ever meet a zero loss scale)."""
    S = roles.shape[0]
    key = torch.zeros(roles.shape[1], dtype=torch.int64, device=roles.device)
    for s in range(S):
        key = key * 3 + roles[s].to(torch.int64)
    return torch.argsort(key, stable=True)


class MfmaOperands:
    """bf16 hi/lo operand copies of one dataset for the MFMA objective, built once and kept
    resident next to the fp32 X (8 more bytes per element; 10M x 1000 -> 82 GB of the
    288 GB HBM): ``X`` (forward A operand, K = features padded to 32) and ``X^T`` with a row
    of ones appended (gradient B operand, K = rows; the ones row yields the intercept
    gradient), both in the kernel's K-tiled layout ``[K/32, rows, 32]``.

    Fold-grouped rows (``DML_LR_FOLD_ROWS``, default on): the operand rows are permuted by
    ``fold_grouped_perm`` of the dataset's split roles, with labels and roles permuted
    alike (``y``, ``roles``).  The objective is a sum over rows, so the order changes no
    term; but each split's rows without a training role now fill whole row tiles, and the
    v3 kernels skip those tiles for that split's fits (``rt_skip``): 5-fold CV spends no
    matrix-core work on the 20 % of rows each fit holds out."""

    def __init__(self, data):
        lib = native.hip_lib()
        n, d, dev = data.n, data.d, data.device
        self.npad = _roundup(n, _ROW_TILE)
        self.Kp = _roundup(d, 32)
        self.Dp = _roundup(d + 1, _TILE)
        bf = torch.bfloat16
        self.xh = torch.zeros((self.Kp // 32, self.npad, 32), dtype=bf, device=dev)
        self.xl = torch.zeros_like(self.xh)
        self.xth = torch.zeros((self.npad // 32, self.Dp, 32), dtype=bf, device=dev)
        self.xtl = torch.zeros_like(self.xth)
        st = native.stream_handle(dev)
        roles = getattr(data, "roles", None)
        self.roles_key = roles.clone() if roles is not None else None   # the split roles this layout is for
        perm = None
        if (roles is not None and roles.shape[0] >= 2 and os.environ.get("DML_LR_FOLD_ROWS", "1") != "0"
                and getattr(data, "y_cls", None) is not None):
            perm = fold_grouped_perm(roles)
        self.perm = perm
        for hi, lo, drows, tr in ((self.xh, self.xl, self.npad, 0), (self.xth, self.xtl, self.Dp, 1)):
            rc = lib.dml_split_hilo(native.ptr(data.X), n, d, d, native.ptr(hi), native.ptr(lo), drows, tr,
                                    native.ptr(perm) if perm is not None else None, st)
            if rc:
                raise RuntimeError(f"dml_split_hilo failed ({rc})")
        ones = torch.zeros(self.npad, dtype=bf, device=dev)
        ones[:n] = 1.0
        self.xth[:, d, :] = ones.view(-1, 32)
        # labels / roles in operand row order, and each split's row tiles without a training row
        self.y = data.y_cls[perm].contiguous() if perm is not None else data.y_cls
        self.roles = roles[:, perm].contiguous() if perm is not None else roles
        self.rt_skip = None
        self.blk32_train = None
        if perm is not None:
            S = roles.shape[0]
            tr = torch.zeros((S, self.npad), dtype=torch.bool, device=dev)
            tr[:, :n] = self.roles == 1
            self.rt_skip = (~tr.view(S, self.npad // _ROW_TILE, _ROW_TILE).any(2)).to(torch.uint8).contiguous()
            # per 32-row block (the K granularity of the gradient's slices), host side
            self.blk32_train = tr.view(S, self.npad // 32, 32).any(2).cpu().numpy()

    def matches(self, data) -> bool:
        roles = getattr(data, "roles", None)
        if self.roles_key is None or roles is None:
            return self.roles_key is None and roles is None
        return self.roles_key.shape == roles.shape and bool(torch.equal(self.roles_key, roles))


def mfma_operands(data) -> MfmaOperands:
    ops = getattr(data, "_lr_mfma_ops", None)
    if ops is not None and not ops.matches(data):   # other split roles: another row grouping
        data._lr_mfma_ops = ops = None
    if ops is None:
        ops = MfmaOperands(data)
        data._lr_mfma_ops = ops
    return ops


class MfmaPlan:
    """Buffers and launch blocks of one batch's matrix-core objective
    (csrc/kernels/lr_mfma.hip): forward GEMM + fused link epilogue writing R^T, then the
    split-K gradient GEMM into per-slice slabs (summed here in a fixed order)."""

    def __init__(self, data, b: "_Batch"):
        lib = native.hip_lib()
        if lib.dml_lr_mfma_tile() != _TILE:
            raise RuntimeError("lr_mfma tile mismatch")
        self.ops = ops = mfma_operands(data)
        dev = data.device
        # padded column layout: no fit's column group straddles a 128-column tile.  Fits are
        # laid out by (objective, C): fits that stop at similar iterations share column tiles,
        # so the tiles of stopped fits empty out and the kernels skip them (``live`` below)
        def _order_key(f):
            rp = b.tasks[f].params
            return (bool(rp.get("penalize_intercept")), float("inf") if rp.get("C") is None else float(rp["C"]))

        def layout(by_split: bool):
            # by_split: fits of one split are contiguous and a split starts a 256-column m tile
            # (fold-grouped rows: a tile of one split can skip that split's held-out row tiles)
            pc, m_, prev = [0] * len(b.K_l), 0, None
            key = (lambda f: (b.split_l[f],) + _order_key(f)) if by_split else _order_key
            for f in sorted(range(len(b.K_l)), key=key):
                k = b.K_l[f]
                if by_split and prev is not None and b.split_l[f] != prev:
                    m_ = _roundup(m_, _ROW_TILE)
                prev = b.split_l[f]
                if (m_ % _TILE) + k > _TILE:
                    m_ = _roundup(m_, _TILE)
                pc[f] = m_
                m_ += k
            return pc, m_

        pcol0, m = layout(False)
        self.v3 = lr_v3(lib, m)
        self.by_split = False
        if self.v3 and ops.rt_skip is not None and len(set(b.split_l)) > 1:
            pg, mg = layout(True)
            if _roundup(mg, _ROW_TILE) <= 1.1 * _roundup(m, _ROW_TILE):   # padding costs < 10 %
                pcol0, m, self.by_split = pg, mg, True
        if self.v3 and lib.dml_lr_v3_row_tile() != _ROW_TILE:
            raise RuntimeError("lr_mfma v3 row tile mismatch")
        self.Mp = _roundup(max(m, 1), _ROW_TILE if self.v3 else _TILE)
        col_tiles = self.Mp // _TILE
        self.colmap = torch.tensor([c0 + j for c0, k in zip(pcol0, b.K_l) for j in range(k)], dtype=torch.long,
                                   device=dev)
        self.col_fit = torch.full((self.Mp,), -1, dtype=torch.int32, device=dev)
        self.col_fit[self.colmap] = b.col_fit.to(torch.int32)
        self.fit_col0 = torch.tensor(pcol0, dtype=torch.int32, device=dev)
        bf = torch.bfloat16
        self.w_lin = torch.zeros((2, self.Mp, ops.Kp), dtype=bf, device=dev)     # hi/lo, row-major
        self.wh = torch.zeros((ops.Kp // 32, self.Mp, 32), dtype=bf, device=dev)  # K-tiled copies
        self.wl = torch.zeros_like(self.wh)
        self.bias = torch.zeros(self.Mp, dtype=torch.float32, device=dev)
        self.loss = torch.zeros(b.F, dtype=torch.float64, device=dev)
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        self.lpart = self.col_info = self.col_scale = None
        self.softmax_any = any(kd == KIND_SOFTMAX for kd in b.kind_l)
        n_tiles = ops.Dp // _TILE
        p = native.ptr
        if self.v3:
            # per padded column: kind << 28 | split << 16 | positive class (OvR column j: class j),
            # -1 on padding; and the fit's loss scale (k_lr_fwd3's register epilogue)
            info = np.full(self.Mp, -1, dtype=np.int64)
            cscale = np.zeros(self.Mp, dtype=np.float32)
            sc_host = b.scale.cpu().numpy()
            for f, (c0, k, kd, sp) in enumerate(zip(pcol0, b.K_l, b.kind_l, b.split_l)):
                if sp >= 4096:
                    raise RuntimeError("lr_mfma v3: split index out of range")
                for j in range(k):
                    info[c0 + j] = (kd << 28) | (sp << 16) | (j if kd == KIND_OVR else 1)
                    cscale[c0 + j] = sc_host[f]
            self.col_info = torch.from_numpy(info.astype(np.int32)).to(dev)
            self.col_scale = torch.from_numpy(cscale).to(dev)
            self.k_uniform = len(set(b.K_l)) == 1
            # ROW CHUNKS: the residual R^T exists for one chunk of rows at a time (forward of the
            # chunk, then the chunk's split-K gradient into its own slabs), so a batch's memory is
            # R^T of one chunk (<= DML_LR_RT_GB, default 16 GB) instead of 4 bytes per (row, column)
            # of the whole table -- every fit of a config-4 search fits ONE batch
            rt_budget = float(os.environ.get("DML_LR_RT_GB", "16")) * 2 ** 30
            chunk = max(_ROW_TILE, int(rt_budget // (4 * self.Mp)) // _ROW_TILE * _ROW_TILE)
            chunk = min(chunk, ops.npad)
            self.n_chunks = -(-ops.npad // chunk)
            self.rh = torch.zeros((chunk // 32, self.Mp, 32), dtype=bf, device=dev)   # pad columns stay 0
            self.rl = torch.zeros_like(self.rh)
            self.lpart = torch.empty((ops.npad // _ROW_TILE, self.Mp), dtype=torch.float64, device=dev)
            m_tiles = self.Mp // _ROW_TILE
            tiles = m_tiles * n_tiles
            # column tiles still holding an active fit: [n_live, tile ids...] (forward) and one
            # flag per 256-column gradient tile; set on the device each evaluation (no host sync)
            self.live = torch.cat([torch.tensor([col_tiles], dtype=torch.int32),
                                   torch.arange(col_tiles, dtype=torch.int32)]).to(dev)
            self.mlive = torch.ones(m_tiles, dtype=torch.int32, device=dev)
            self.skip_done = os.environ.get("DML_LR_SKIP_DONE", "1") != "0"
            S = _roundup(-(-4 * cus // tiles), 8)              # >= ~4 waves of workgroups per chunk
            Kc = _roundup(-(-chunk // S), 32)
            S = _roundup(-(-chunk // Kc), 8)
            # fold-grouped rows: the split of every column tile / m tile (-1 mixed or none), and
            # per row chunk the gradient slices without a training row of the m tile's split
            self.ct_split = self.kskip_l = None
            if self.by_split:
                cts = np.full(col_tiles, -2, dtype=np.int64)   # -2: no fit column
                for f, (c0, k) in enumerate(zip(pcol0, b.K_l)):
                    for ct in {c0 // _TILE, (c0 + k - 1) // _TILE}:
                        cts[ct] = b.split_l[f] if cts[ct] in (-2, b.split_l[f]) else -1
                mts = np.full(m_tiles, -1, dtype=np.int64)
                for mt in range(m_tiles):
                    vals = {int(v) for v in cts[2 * mt:2 * mt + 2] if v != -2}
                    mts[mt] = vals.pop() if len(vals) == 1 else -1
                self.ct_split = torch.from_numpy(np.where(cts == -2, -1, cts).astype(np.int32)).to(dev)
                csum = np.concatenate([np.zeros((ops.blk32_train.shape[0], 1), dtype=np.int64),
                                       np.cumsum(ops.blk32_train, axis=1)], axis=1)   # [splits, blocks + 1]
                self.kskip_l = []
                for ci in range(self.n_chunks):
                    r0 = ci * chunk
                    rows_c = min(chunk, ops.npad - r0)
                    ks = np.zeros((m_tiles, S), dtype=np.int32)
                    for mt in range(m_tiles):
                        sp = int(mts[mt])
                        if sp < 0:
                            continue
                        for k in range(S):
                            a0, a1 = r0 + k * Kc, r0 + min((k + 1) * Kc, rows_c)
                            if a1 > a0 and csum[sp, a1 // 32] - csum[sp, a0 // 32] == 0:
                                ks[mt, k] = 1
                    self.kskip_l.append(torch.from_numpy(ks).to(dev))
            self.slabs = torch.empty((self.n_chunks * S, self.Mp, ops.Dp), dtype=torch.float32, device=dev)
            rg = max(8, cus // 8 * 8)   # forward: one persistent workgroup per CU
            self.fwd_l, self.grad_l = [], []
            for ci in range(self.n_chunks):
                r0 = ci * chunk
                rows_c = min(chunk, ops.npad - r0)
                self.fwd_l.append(native.LrFwdArgs(
                    xh=p(ops.xh), xl=p(ops.xl), xrows=ops.npad, wh=p(self.wh), wl=p(self.wl), n=data.n, Kp=ops.Kp,
                    row_tiles=rows_c // _ROW_TILE, col_tiles=col_tiles, row_groups=rg, bias=p(self.bias),
                    col_fit=p(self.col_fit), fit_col0=p(self.fit_col0), fit_k=p(b.K), fit_kind=p(b.kind),
                    fit_split=p(b.split), scale=p(b.scale), cw=p(b.cw),
                    cwC=int(b.cw.shape[1]) if b.cw is not None else 0, y=p(ops.y), roles=p(ops.roles),
                    rh=p(self.rh), rl=p(self.rl), kr=rows_c, loss=p(self.loss), lpart=p(self.lpart),
                    col_info=p(self.col_info), col_scale=p(self.col_scale), n_splits=int(data.roles.shape[0]),
                    softmax_any=int(self.softmax_any), row_base=r0 // _ROW_TILE, live=p(self.live),
                    ct_split=p(self.ct_split), rt_skip=p(ops.rt_skip) if self.by_split else 0,
                    rt_stride=ops.npad // _ROW_TILE))
                self.grad_l.append(native.LrGradArgs(
                    rh=p(self.rh), rl=p(self.rl), unused=0, xth=p(ops.xth), xtl=p(ops.xtl), m_tiles=m_tiles,
                    n_tiles=n_tiles, Kp=rows_c, S=S, Kc=Kc, out=p(self.slabs), bk_off=r0, slab0=ci * S,
                    mlive=p(self.mlive), kskip=p(self.kskip_l[ci]) if self.kskip_l else 0))
        else:
            self.rh = torch.zeros((ops.npad // 32, self.Mp, 32), dtype=bf, device=dev)   # pad columns stay 0
            self.rl = torch.zeros_like(self.rh)
            # forward: persistent, at most the resident workgroups (2 per CU), row groups % 8 == 0
            row_tiles = ops.npad // _TILE
            resident = 2 * cus
            rg = max(8, (resident // col_tiles) // 8 * 8)
            rg = min(rg, _roundup(row_tiles, 8))
            # gradient: output tiles x K slices >= ~4 waves of workgroups; slices % 8 == 0
            tiles = col_tiles * n_tiles
            S = _roundup(-(-4 * resident // tiles), 8)
            Kc = _roundup(-(-ops.npad // S), 32)
            S = _roundup(-(-ops.npad // Kc), 8)
            self.slabs = torch.empty((S, self.Mp, ops.Dp), dtype=torch.float32, device=dev)
            self.fwd = native.LrFwdArgs(
                xh=p(ops.xh), xl=p(ops.xl), xrows=ops.npad, wh=p(self.wh), wl=p(self.wl), n=data.n, Kp=ops.Kp,
                row_tiles=row_tiles, col_tiles=col_tiles, row_groups=rg, bias=p(self.bias), col_fit=p(self.col_fit),
                fit_col0=p(self.fit_col0), fit_k=p(b.K), fit_kind=p(b.kind), fit_split=p(b.split), scale=p(b.scale),
                cw=p(b.cw), cwC=int(b.cw.shape[1]) if b.cw is not None else 0, y=p(ops.y), roles=p(ops.roles),
                rh=p(self.rh), rl=p(self.rl), kr=ops.npad, loss=p(self.loss))
            self.grad = native.LrGradArgs(
                rh=p(self.rh), rl=p(self.rl), unused=0, xth=p(ops.xth), xtl=p(ops.xtl), m_tiles=col_tiles,
                n_tiles=n_tiles, Kp=ops.npad, S=S, Kc=Kc, out=p(self.slabs))
        self.fit_col0_l = self.fit_col0.long()
        self.zero_groups = _zero_groups(data, b)   # the solver's W = 0 start (LogisticFamily._objective_at_zero)

    def set_active(self, b: "_Batch", active: Optional[torch.Tensor]):
        """Mark the column tiles whose fits have all stopped (v3 kernels skip them; the
        solver only reads the loss / gradient of active fits)."""
        if not self.v3:
            return
        col_tiles = self.Mp // _TILE
        if active is None or not self.skip_done:
            self.live[0] = col_tiles
            self.live[1:] = torch.arange(col_tiles, dtype=torch.int32, device=self.live.device)
            self.mlive.fill_(1)
            return
        colact = torch.zeros(self.Mp, dtype=torch.bool, device=active.device)
        colact[self.colmap] = active[b.col_fit]
        tl = colact.view(col_tiles, _TILE).any(1)
        self.live[0] = tl.sum().to(torch.int32)
        self.live[1:] = torch.argsort((~tl).to(torch.int32), stable=True).to(torch.int32)   # live tiles first
        self.mlive.copy_(tl.view(-1, _ROW_TILE // _TILE).any(1).to(torch.int32))

    def objective(self, data, b: "_Batch", W: torch.Tensor, active: Optional[torch.Tensor] = None,
                  w_zero: bool = False):
        """(loss [F] float64, data gradient [d+1, M]) of the unregularised objective; with
        ``active``, entries of stopped fits may be stale.  ``w_zero``: the caller knows W == 0
        (the solver's start), so the forward GEMM is skipped (exactly: its result is 0)."""
        d = data.d
        self.set_active(b, active)
        if self.v3:
            for fa in self.fwd_l:
                fa.w_zero = int(w_zero)
        Wt = W[:d].t()
        hi = Wt.to(torch.bfloat16)
        self.w_lin[0, self.colmap, :d] = hi
        self.w_lin[1, self.colmap, :d] = (Wt - hi.float()).to(torch.bfloat16)
        kb = self.w_lin.shape[2] // 32
        self.wh.copy_(self.w_lin[0].view(self.Mp, kb, 32).transpose(0, 1))
        self.wl.copy_(self.w_lin[1].view(self.Mp, kb, 32).transpose(0, 1))
        self.bias[self.colmap] = W[d] * b.icpt_col
        self.loss.zero_()
        lib = native.hip_lib()
        st = native.stream_handle(data.device)
        if self.v3:   # row chunks in order on one stream: chunk c+1's forward reuses R^T after c's gradient
            rc = 0
            for fa, ga in zip(self.fwd_l, self.grad_l):
                rc = lib.dml_lr_mfma_fwd3(ctypes.byref(fa), st)
                if rc == 0:
                    rc = lib.dml_lr_mfma_grad3(ctypes.byref(ga), st)
                if rc:
                    break
        else:
            rc = lib.dml_lr_mfma_fwd(ctypes.byref(self.fwd), st)
            if rc == 0:
                rc = lib.dml_lr_mfma_grad(ctypes.byref(self.grad), st)
        if rc:
            raise RuntimeError(f"lr_mfma launch failed ({rc})")
        if self.v3:
            # every (row tile, column) partial is written once; fixed-order sums over row tiles,
            # then over each fit's columns (OvR: k sigmoid columns; binary / softmax: one)
            colsum = self.lpart.sum(0)[self.colmap]
            if self.k_uniform:
                self.loss.copy_(colsum.view(b.F, -1).sum(1))
            else:
                self.loss.copy_(torch.zeros_like(self.loss).index_add_(0, b.col_fit, colsum))
        GT = self.slabs.sum(0)
        G = torch.empty_like(W)
        G[:d] = GT[self.colmap, :d].t()
        G[d] = GT[self.colmap, d] * b.icpt_col
        return self.loss.clone(), G


def _zero_groups(data, b: "_Batch"):
    """At W = 0 every logit is 0, so fits with the same (split, link, classes, loss scale,
    class weights) have IDENTICAL residual columns.  Returns (sub-batch of one representative
    per group, source column of every batch column, representative of every fit), or None
    when there are too few duplicates to pay (or no resident fp32 rows).  Host-side keys
    only; built with the plan, so the solve itself stays free of host syncs."""
    if os.environ.get("DML_LR_ZERO_DEDUP", "1") == "0" or getattr(b, "streamed", False) or \
            getattr(data, "X", None) is None:
        return None
    groups: Dict[tuple, int] = {}
    rep = []
    for f in range(b.F):
        key = (b.split_l[f], b.kind_l[f], b.K_l[f], b.scale_l[f], repr(b.tasks[f].params.get("class_weight")))
        rep.append(groups.setdefault(key, len(groups)))
    if len(groups) * 4 > b.F:
        return None
    reps = [0] * len(groups)
    for f in reversed(range(b.F)):
        reps[rep[f]] = f
    sub = _Batch(data, [b.tasks[f] for f in reps])
    dev = data.device
    src = torch.tensor([sub.col0_l[rep[f]] + j for f in range(b.F) for j in range(b.K_l[f])],
                       dtype=torch.long, device=dev)
    return sub, src, torch.tensor(rep, dtype=torch.long, device=dev)


class _Batch:
    """Column layout of a batch of logistic fits."""

    def __init__(self, data, tasks: List[FitTask]):
        self.tasks = tasks
        self.mf = None   # MfmaPlan when the matrix-core objective runs
        C = data.n_classes
        col0, K, kind, split, scale, lam, lam1, icpt, pen_icpt, tol, max_iter, cws = ([] for _ in range(12))
        any_cw = False
        m = 0
        for t in tasks:
            rp = t.params
            if C == 2:
                k, kd = 1, KIND_BINARY
            elif rp["ovr"]:
                k, kd = C, KIND_OVR
            else:
                k, kd = C, KIND_SOFTMAX
            n_f = max(1, data.train_counts[t.split])
            cwv = class_weight_vector(data, t.split, rp.get("class_weight"))
            if cwv is not None:
                n_f = float(_dp_sum(data, cwv[data.y_cls[data.train_rows[t.split].long()].long()].sum()))   # sw_sum
                any_cw = True
            cws.append(cwv)
            col0.append(m); K.append(k); kind.append(kd); split.append(t.split)
            scale.append(1.0 / n_f)
            strength = 0.0 if rp["C"] is None else 1.0 / (rp["C"] * n_f)
            l1r = rp.get("l1_ratio", 0.0)
            lam.append(strength * (1.0 - l1r))
            lam1.append(strength * l1r)
            icpt.append(rp["intercept_scaling"] if rp["fit_intercept"] else 0.0)
            pen_icpt.append(1.0 if rp["penalize_intercept"] else 0.0)
            tol.append(rp["tol"]); max_iter.append(rp["max_iter"])
            m += k
        dev = data.device
        self.M, self.F = m, len(tasks)
        i32 = lambda v: torch.tensor(v, dtype=torch.int32, device=dev)
        self.col0_l, self.K_l, self.kind_l, self.split_l = col0, K, kind, split
        self.col0, self.K, self.kind, self.split = i32(col0), i32(K), i32(kind), i32(split)
        self.scale_l = scale
        self.scale = torch.tensor(scale, dtype=torch.float32, device=dev)
        self.col_fit = torch.repeat_interleave(torch.arange(self.F, device=dev), torch.tensor(K, device=dev))
        lam_t = torch.tensor(lam, dtype=torch.float32, device=dev)
        self.lam_col = lam_t[self.col_fit]
        self.l1_col = torch.tensor(lam1, dtype=torch.float32, device=dev)[self.col_fit]
        self.has_l1 = any(v > 0 for v in lam1)
        self.cw = None
        if any_cw:
            ones = torch.ones(C if C > 2 else 2, dtype=torch.float32, device=dev)
            self.cw = torch.stack([ones if v is None else v.float() for v in cws]).contiguous()   # [F, C]
        self.icpt_col = torch.tensor(icpt, dtype=torch.float32, device=dev)[self.col_fit]
        self.pen_icpt_col = torch.tensor(pen_icpt, dtype=torch.float32, device=dev)[self.col_fit]
        self.tol = torch.tensor(tol, dtype=torch.float32, device=dev)
        self.max_iter = torch.tensor(max_iter, dtype=torch.int64, device=dev)

    def segsum(self, v: torch.Tensor) -> torch.Tensor:
        out = torch.zeros(self.F, dtype=v.dtype, device=v.device)
        return out.index_add_(0, self.col_fit, v)

    def segmax(self, v: torch.Tensor) -> torch.Tensor:
        out = torch.zeros(self.F, dtype=v.dtype, device=v.device)
        return out.scatter_reduce_(0, self.col_fit, v, reduce="amax", include_self=True)


class LogisticFamily(Family):
    model_types = ("LogisticRegression",)
    classifiers = ("LogisticRegression",)
    history = 10
    data_parallel = True   # loss + gradient all-reduced per objective evaluation under a RowShard
    # binned-only tables (float32 rows too large for HBM): every objective evaluation is one
    # pass over the host rows in chunks, all candidates x folds of the batch per chunk
    streams_rows = True

    def resolve(self, model_type, params, n_train, n_features, n_classes):
        p = dict(_LR_DEFAULTS)
        p.update({k: v for k, v in params.items() if k in _LR_DEFAULTS})
        warn = []
        unknown = sorted(k for k in params if k not in _LR_DEFAULTS)
        if unknown:
            warn.append(f"ignored unknown parameters {unknown}")
        solver = p["solver"] or "lbfgs"
        if solver not in _SOLVERS:
            raise ParamError(f"solver must be one of {_SOLVERS}, got {solver!r}")
        penalty = p["penalty"]
        if penalty in ("none", "None"):
            penalty = None
        if penalty not in ("l2", None, "l1", "elasticnet"):
            raise ParamError(f"penalty {penalty!r} invalid")
        l1_ratio = 0.0
        if penalty == "l1":
            if solver not in ("liblinear", "saga"):
                raise ParamError(f"Solver {solver} supports only 'l2' or None penalties, got l1 penalty.")
            l1_ratio = 1.0
        elif penalty == "elasticnet":
            if solver != "saga":
                raise ParamError(f"Only 'saga' solver supports elasticnet penalty, got solver={solver}.")
            if p["l1_ratio"] is None:
                raise ParamError("l1_ratio must be specified when penalty is elasticnet.")
            l1_ratio = as_float(p["l1_ratio"], "l1_ratio", lo=0.0, hi=1.0)
        if penalty is None and solver == "liblinear":
            raise ParamError("penalty=None is not supported for the liblinear solver")
        C = as_float(p["C"], "C", lo=0.0)
        if C <= 0:
            raise ParamError("Penalty term must be positive")
        mc = p["multi_class"]
        ovr = solver == "liblinear" or mc == "ovr"
        cw = p["class_weight"]
        if cw in ("None",):
            cw = None
        if cw is not None and cw != "balanced" and not isinstance(cw, dict):
            raise ParamError("class_weight must be None, 'balanced' or a dict")
        if as_bool(p["dual"], "dual"):
            warn.append("dual=True solved in the primal (same optimum)")
        return {
            "C": None if penalty is None else C,
            "l1_ratio": l1_ratio,
            "class_weight": cw,
            "tol": as_float(p["tol"], "tol", lo=0.0),
            "max_iter": as_int(p["max_iter"], "max_iter", lo=0),
            "fit_intercept": as_bool(p["fit_intercept"], "fit_intercept"),
            "intercept_scaling": as_float(p["intercept_scaling"], "intercept_scaling", lo=0.0)
            if solver == "liblinear" else 1.0,
            "penalize_intercept": solver == "liblinear",
            "ovr": ovr,
            "solver": solver,
            "seed": seed_of(p["random_state"]),
            "warnings": warn,
        }

    def cost(self, model_type, rp, n_train, n_features, n_classes) -> float:
        return max(1, rp["max_iter"]) * n_train * (n_features + 1) * max(1, n_classes - 1) * 4e-12 + 1e-3

    # --------------------------------------------------------------------------------
    def _objective(self, data, b: _Batch, W: torch.Tensor, active: Optional[torch.Tensor] = None,
                   w_zero: bool = False):
        d = data.d
        if getattr(b, "streamed", False):
            return self._objective_streamed(data, b, W)
        if b.mf is not None:   # matrix cores: fused forward + split-K gradient (lr_mfma.hip)
            loss, G = b.mf.objective(data, b, W, active, w_zero)
            loss, G = _dp_sum(data, loss), _dp_sum(data, G)
            reg = W * b.lam_col
            reg[d] = reg[d] * b.pen_icpt_col
            G += reg
            return loss + 0.5 * b.segsum((W * reg).sum(0)).double(), G
        X = data.X
        Z = torch.addmm(W[d] * b.icpt_col, X, W[:d])
        if data.is_gpu:
            R = torch.empty_like(Z)
            loss = torch.empty(b.F, dtype=torch.float64, device=Z.device)
            lib = native.hip_lib()
            rc = lib.dml_lr_link_grad(native.ptr(Z), data.n, b.M, native.ptr(data.y_cls), native.ptr(data.roles),
                                      native.ptr(b.col0), native.ptr(b.K), native.ptr(b.kind), native.ptr(b.split),
                                      native.ptr(b.scale), b.F, native.ptr(b.cw), int(b.cw.shape[1]) if b.cw is not None
                                      else 0, native.ptr(R), native.ptr(loss), native.stream_handle(data.device))
            if rc:
                raise RuntimeError("dml_lr_link_grad failed")
        else:
            R, loss = link_grad_torch(Z, data.y_cls, data.roles, b.col0_l, b.K_l, b.kind_l, b.split_l, b.scale.tolist(),
                                      b.cw)
        G = torch.empty_like(W)
        G[:d] = X.t() @ R
        G[d] = R.sum(0) * b.icpt_col
        loss, G = _dp_sum(data, loss), _dp_sum(data, G)
        reg = W * b.lam_col
        reg[d] = reg[d] * b.pen_icpt_col
        G += reg
        f = loss + 0.5 * b.segsum((W * reg).sum(0)).double()
        return f, G

    @staticmethod
    def _link_grad(data, b: _Batch, Z: torch.Tensor, y: torch.Tensor, roles: torch.Tensor):
        """(R, loss[F]) of logits Z over the rows of y / roles (the fused kernel on the GPU)."""
        if not data.is_gpu:
            return link_grad_torch(Z, y, roles, b.col0_l, b.K_l, b.kind_l, b.split_l, b.scale.tolist(), b.cw)
        n = Z.shape[0]
        R = torch.empty_like(Z)
        loss = torch.empty(b.F, dtype=torch.float64, device=Z.device)
        rc = native.hip_lib().dml_lr_link_grad(
            native.ptr(Z), n, b.M, native.ptr(y), native.ptr(roles), native.ptr(b.col0), native.ptr(b.K),
            native.ptr(b.kind), native.ptr(b.split), native.ptr(b.scale), b.F, native.ptr(b.cw),
            int(b.cw.shape[1]) if b.cw is not None else 0, native.ptr(R), native.ptr(loss),
            native.stream_handle(data.device))
        if rc:
            raise RuntimeError("dml_lr_link_grad failed")
        return R, loss

    def _objective_streamed(self, data, b: _Batch, W: torch.Tensor):
        """The objective over a binned-only table: the host rows stream through in chunks
        (DeviceData.stream_rows), each chunk's logits, link gradient and X^T R accumulate
        into one loss / gradient -- one pass over the table per evaluation, every fit of the
        batch at once (the same link kernel as the resident path, chunk by chunk)."""
        d = data.d
        loss = torch.zeros(b.F, dtype=torch.float64, device=data.device)
        G = torch.zeros_like(W)
        bias = W[d] * b.icpt_col
        for r0, r1, Xc in data.stream_rows(_lr_stream_chunk(data, b.M)):
            Zc = torch.addmm(bias, Xc, W[:d])
            Rc, lc = self._link_grad(data, b, Zc, data.y_cls[r0:r1].contiguous(), data.roles[:, r0:r1].contiguous())
            loss += lc
            G[:d] += Xc.t() @ Rc
            G[d] += Rc.sum(0) * b.icpt_col
        reg = W * b.lam_col
        reg[d] = reg[d] * b.pen_icpt_col
        G += reg
        return loss + 0.5 * b.segsum((W * reg).sum(0)).double(), G

    def _objective_at_zero(self, data, b: _Batch):
        """The objective at the solver's start W = 0 from one representative fit per residual
        group (``_zero_groups``; a config-4 search has 5 groups for 2,560 fits): one fp32 GEMM
        of X^T against a handful of columns, the group's loss / gradient columns copied to its
        fits.  None when grouping does not pay."""
        zg = b.mf.zero_groups if b.mf is not None else _zero_groups(data, b)
        if zg is None:
            return None
        sub, src, rep_t = zg
        d, dev = data.d, data.device
        Z = torch.zeros((data.X.shape[0], sub.M), dtype=torch.float32, device=dev)
        R, loss_s = self._link_grad(data, sub, Z, data.y_cls, data.roles)
        GTs = data.X.t() @ R
        G = torch.empty((d + 1, b.M), dtype=torch.float32, device=dev)
        G[:d] = GTs[:, src]
        G[d] = R.sum(0)[src] * b.icpt_col
        return _dp_sum(data, loss_s[rep_t]), _dp_sum(data, G)      # the penalty is 0 at W = 0

    def _solve(self, data, b: _Batch):
        """Batched L-BFGS that stays on the device; columns with an L1 term use OWL-QN
        (Andrew & Gao 2007): pseudo-gradient, orthant-constrained direction and line
        search.  Columns without L1 reduce exactly to plain L-BFGS.

        Every fit runs its own L-BFGS state machine, advanced by masked tensor ops: one
        global step = one batched objective evaluation at every fit's current trial point,
        after which each fit independently accepts its trial (Armijo; history push into
        its slot of a ring buffer, new two-loop direction, step 1) or backtracks (halve its
        step).  A fit that backtracks therefore never holds the others back, and nothing on
        the way needs the host: the only device->host read is the "any fit still active"
        flag, once every ``sync_every`` steps (``last_solve_stats['host_syncs']``).  Each
        fit's iterates are the ones a lock-step L-BFGS would produce for it alone."""
        d, dev = data.d, data.device
        H, Fn = self.history, b.F
        col = b.col_fit
        W = torch.zeros((d + 1, b.M), dtype=torch.float32, device=dev)
        start = self._objective_at_zero(data, b) if b.mf is not None else None
        f, G = start if start is not None else self._objective(data, b, W, w_zero=True)
        l1 = None
        if b.has_l1:
            l1 = b.l1_col.view(1, -1).repeat(d + 1, 1)
            l1[d] = l1[d] * b.pen_icpt_col                     # intercept: L1 only when penalised (liblinear)
            l1on = l1 > 0

        def total(fv, Wv):
            return fv if l1 is None else fv + b.segsum((l1 * Wv.abs()).sum(0)).double()

        def pseudo(Wv, Gv):
            if l1 is None:
                return Gv
            gp, gm = Gv + l1, Gv - l1
            at0 = torch.where(gp < 0, gp, torch.where(gm > 0, gm, torch.zeros_like(Gv)))
            return torch.where(Wv != 0, Gv + l1 * torch.sign(Wv), at0)

        S = torch.zeros((H, d + 1, b.M), dtype=W.dtype, device=dev)   # ring buffers of (s, y) pairs
        Y = torch.zeros_like(S)
        RHO = torch.zeros((H, Fn), dtype=torch.float32, device=dev)
        hcount = torch.zeros(Fn, dtype=torch.int64, device=dev)       # pairs pushed per fit
        iters = torch.zeros(Fn, dtype=torch.int64, device=dev)
        stalled = torch.zeros(Fn, dtype=torch.bool, device=dev)
        ls = torch.zeros(Fn, dtype=torch.int32, device=dev)           # trials of the current iteration
        step = torch.ones(Fn, dtype=torch.float32, device=dev)
        hidx = torch.arange(H, device=dev)

        def direction(PGv, Wv, act):
            """Two-loop recursion over each fit's own newest-first history; returns the
            search direction and (OWL-QN) the orthant signs of the line search."""
            q = PGv.clone()
            n_hist = hcount.clamp(max=H)
            slots, alphas = [], []
            for i in range(H):
                slot = (hcount - 1 - i) % H                            # [F]
                valid = (i < n_hist).to(RHO.dtype)
                sl_col = slot[col].view(1, 1, -1).expand(1, d + 1, b.M)
                Si, Yi = S.gather(0, sl_col)[0], Y.gather(0, sl_col)[0]
                rho_i = RHO.gather(0, slot.view(1, -1))[0] * valid
                a_i = rho_i * b.segsum((Si * q).sum(0))
                q -= a_i[col] * Yi
                slots.append((Si, Yi, rho_i))
                alphas.append(a_i)
            S0, Y0, _ = slots[0]
            sy = b.segsum((S0 * Y0).sum(0))
            yy = b.segsum((Y0 * Y0).sum(0))
            gamma_h = torch.where(yy > 0, sy / yy.clamp_min(1e-30), torch.ones_like(yy))
            gnorm = b.segsum((PGv * PGv).sum(0)).sqrt()
            gamma = torch.where(hcount > 0, gamma_h, 1.0 / gnorm.clamp_min(1.0))
            r = q * gamma[col]
            for i in reversed(range(H)):
                Si, Yi, rho_i = slots[i]
                bb = rho_i * b.segsum((Yi * r).sum(0))
                r += (alphas[i] - bb)[col] * Si
            act_col = act[col].to(Wv.dtype)
            p = -r * act_col
            if l1 is not None:   # keep the direction in the pseudo-gradient's orthant
                p = torch.where(l1on & (p * PGv >= 0), torch.zeros_like(p), p)
            gtp = b.segsum((PGv * p).sum(0))
            bad = ((gtp >= 0) & act)[col].unsqueeze(0)               # not a descent direction:
            p = torch.where(bad, -PGv * act_col, p)                  # restart from steepest descent
            xi = None if l1 is None else torch.where(Wv != 0, torch.sign(Wv), torch.sign(-PGv))
            return p, xi

        def trial(Wv, p, xi, stp, act):
            Wt = Wv + p * stp[col]
            if xi is not None:   # orthant projection
                Wt = torch.where(l1on & (Wt * xi <= 0), torch.zeros_like(Wt), Wt)
            return torch.where(act[col].unsqueeze(0), Wt, Wv)

        Ftot = total(f, W)
        PG = pseudo(W, G)
        active = (b.segmax(PG.abs().amax(0)) > b.tol) & (iters < b.max_iter)
        P, XI = direction(PG, W, active)
        Wt = trial(W, P, XI, step, active)
        max_it = max((t.params["max_iter"] for t in b.tasks), default=0)
        sync_every = max(1, int(os.environ.get("DML_LR_SYNC_EVERY", "4")))
        n_evals, host_syncs, steps = 1, 0, 0
        if max_it > 0:
            host_syncs += 1
            running = bool(active.any())
        else:
            running = False
        max_steps = max_it * 31
        # DML_LR_TRACE_ACTIVE=1: active fits per step (device scalars, read once at the end --
        # one extra host sync, so diagnostics only)
        act_hist = [] if os.environ.get("DML_LR_TRACE_ACTIVE") == "1" else None
        while running and steps < max_steps:
            if act_hist is not None:
                act_hist.append(active.sum())
            ft, Gt = self._objective(data, b, Wt, active)
            Ft = total(ft, Wt)
            n_evals += 1
            steps += 1
            # float32 (or bf16x3 on the matrix cores) objective: tolerate round-off near the optimum
            slack = (4e-6 if b.mf is not None else 1e-7) * Ftot.abs() + 1e-12
            dec = b.segsum((PG * (Wt - W)).sum(0)).double()
            ok = Ft <= Ftot + 1e-4 * dec + slack
            acc = ok & active
            rej = active & ~ok
            ls = ls + rej.to(ls.dtype)
            fail = rej & (ls >= 30)                                  # line search exhausted
            stalled |= fail
            # accepted fits push (s, y) into their next ring slot and move to the trial point
            acc_c = acc[col].unsqueeze(0)
            s_vec = Wt - W
            y_vec = Gt - G
            sy = b.segsum((s_vec * y_vec).sum(0))
            rho = torch.where(sy > 1e-10, 1.0 / sy.clamp_min(1e-10), torch.zeros_like(sy))
            slot = hcount % H
            put = (hidx.view(-1, 1) == slot.view(1, -1)) & acc.view(1, -1)     # [H, F]
            put_c = put[:, col].unsqueeze(1)                                    # [H, 1, M]
            S = torch.where(put_c, s_vec.unsqueeze(0), S)
            Y = torch.where(put_c, y_vec.unsqueeze(0), Y)
            RHO = torch.where(put, rho.view(1, -1), RHO)
            hcount = hcount + acc.to(hcount.dtype)
            W = torch.where(acc_c, Wt, W)
            G = torch.where(acc_c, Gt, G)
            Ftot = torch.where(acc, Ft, Ftot)
            iters = iters + (acc | fail).to(iters.dtype)
            PG = pseudo(W, G)
            active = (b.segmax(PG.abs().amax(0)) > b.tol) & (iters < b.max_iter) & ~stalled
            # accepted fits: new direction at step 1; rejected ones: halve their step
            fresh = acc & active
            Pn, XIn = direction(PG, W, fresh)
            fresh_c = fresh[col].unsqueeze(0)
            P = torch.where(fresh_c, Pn, P)
            if XI is not None:
                XI = torch.where(fresh_c, XIn, XI)
            step = torch.where(fresh, torch.ones_like(step), torch.where(rej, step * 0.5, step))
            ls = torch.where(fresh, torch.zeros_like(ls), ls)
            Wt = trial(W, P, XI, step, active)
            if steps % sync_every == 0:
                host_syncs += 1
                running = bool(active.any())
        self.last_solve_stats = {"host_syncs": host_syncs + bool(act_hist), "steps": steps, "sync_every": sync_every}
        if act_hist:
            self.last_solve_stats["active_per_step"] = torch.stack(act_hist).tolist()
        return W, iters, n_evals

    def run(self, data, tasks: List[FitTask], keep_models: bool = False) -> List[FitOutput]:
        if not tasks:
            return []
        if not data.classification:
            raise ParamError("LogisticRegression needs a classification target")
        # tiny lbfgs problems (iris-sized): a device launch per objective evaluation is pure
        # latency, so they run on the host with scipy's L-BFGS-B on sklearn's exact float64
        # objective -> same iterates as sklearn even where max_iter stops before convergence
        streamed = data.X is None and getattr(data, "can_stream_rows", lambda: False)()
        if data.X is None and not streamed:
            raise ParamError("LogisticRegression needs the float32 rows (this table arrived as bins only)")
        small = [t for t in tasks if t.params["solver"] == "lbfgs" and not getattr(data, "is_row_shard", False) and
                 not streamed and
                 data.train_counts[t.split] * (data.d + 1) * max(1, data.n_classes - 1) <= HOST_LBFGS_MAX_WORK]
        if small:
            done = {o.task_id: o for o in self._run_host_lbfgs(data, small, keep_models)}
            rest = [t for t in tasks if t.task_id not in done]
            if rest:
                done.update({o.task_id: o for o in self.run(data, rest, keep_models)})
            return [done[t.task_id] for t in tasks]
        # memory-budgeted batches of whole fits: Z and R are [n, columns] and the L-BFGS
        # history holds 2 x history [d+1, columns] matrices
        width = 1 if data.n_classes == 2 else data.n_classes
        use_mf = mfma_enabled(data) and not streamed
        if use_mf:   # resident bf16 operands first, so the budget below sees them
            ops = mfma_operands(data)
            if lr_v3(native.hip_lib(), len(tasks) * width):
                # row-chunked objective: R^T of one chunk (DML_LR_RT_GB) is a fixed cost, not per column
                per_col = 4.0 * ((data.d + 1) * (2 * self.history + 10) + 128 * ops.Dp)
            else:
                per_col = 4.0 * (ops.npad + (data.d + 1) * (2 * self.history + 10) + 32 * ops.Dp)
        elif streamed:   # chunk-sized logits / link gradients only
            per_col = 4.0 * (3 * min(data.n, data._chunk_rows) + (data.d + 1) * (2 * self.history + 6))
        else:
            per_col = 4.0 * (3 * data.n + (data.d + 1) * (2 * self.history + 6))
        budget = 0.45 * torch.cuda.mem_get_info(data.device)[0] if data.is_gpu else 8e9
        cap = max(1, int(budget // (per_col * width)))
        if len(tasks) > cap:
            outs: List[FitOutput] = []
            for i in range(0, len(tasks), cap):
                outs.extend(self.run(data, tasks[i:i + cap], keep_models))
            return outs
        t0 = time.perf_counter()
        with trace.range("lr_plan"):
            b = _Batch(data, tasks)
            b.streamed = streamed
            if use_mf:
                b.mf = MfmaPlan(data, b)
        with trace.range("lr_solve"):
            W, iters, n_evals = self._solve(data, b)
        b.mf = None   # release R^T / slabs before the prediction GEMMs
        d = data.d
        with trace.range("lr_test_logits"):
            Zte = self._test_logits(data, b, W)
        iters_h = iters.cpu().tolist()
        self.last_solve_stats["iterations_max"] = max(iters_h, default=0)
        self.last_solve_stats["iterations_hist"] = {int(k): int(v) for k, v in
                                                    zip(*np.unique(np.asarray(iters_h, dtype=np.int64), return_counts=True))}
        self.last_solve_stats["evals"] = int(n_evals)
        outs = []
        # binary fits: every fit of a split predicted by ONE threshold over the split's logit
        # block (not a handful of launches per fit -- 2,560 fits spent ~0.3 s in them);
        # probabilities only when the scorer or the caller needs them
        want_proba = any(getattr(t, "need_proba", False) for t in tasks)
        bin_pred: Dict[int, torch.Tensor] = {}
        if not want_proba and all(kd == KIND_BINARY for kd in b.kind_l):
            by_base: Dict[int, List[int]] = {}
            for f in range(b.F):
                by_base.setdefault(Zte[f].untyped_storage().data_ptr(), []).append(f)   # one block per split
            for fits in by_base.values():
                zs = torch.stack([Zte[f][:, 0] for f in fits])                  # [fits, m]
                pz = (zs > 0).to(torch.int32)
                for i, f in enumerate(fits):
                    bin_pred[f] = pz[i]
        for f, t in enumerate(tasks):
            k = b.K_l[f]
            z = Zte[f]
            if b.kind_l[f] == KIND_BINARY:
                if f in bin_pred:
                    pred, proba = bin_pred[f], None
                else:
                    pred = (z[:, 0] > 0).to(torch.int32)
                    proba = torch.sigmoid(z[:, 0])
                    proba = torch.stack([1 - proba, proba], 1)
            else:
                pred = z.argmax(1).to(torch.int32)
                proba = torch.softmax(z, 1) if b.kind_l[f] == KIND_SOFTMAX else None
                if proba is None:
                    pz = torch.sigmoid(z)
                    proba = pz / pz.sum(1, keepdim=True).clamp_min(1e-30)
            outs.append(FitOutput(task_id=t.task_id, pred=pred, proba=proba,
                                  info={"warnings": t.params.get("warnings", []), "n_iter": int(iters_h[f])}))
        if data.is_gpu:
            torch.cuda.synchronize(data.device)
        dt = time.perf_counter() - t0
        for o in outs:
            o.fit_seconds = dt / len(outs)
            o.info["objective_evals"] = n_evals
        if keep_models:
            for f, (o, t) in enumerate(zip(outs, tasks)):
                c0, k = b.col0_l[f], b.K_l[f]
                o.model = {
                    "kind": "linear_logistic", "coef": W[:d, c0:c0 + k].t().cpu().numpy(),
                    "intercept": (W[d, c0:c0 + k] * b.icpt_col[c0:c0 + k]).cpu().numpy(),
                    "link": b.kind_l[f], "classes": np.asarray(data.classes).tolist(),
                    "model_type": t.model_type, "params": {k2: v for k2, v in t.params.items() if k2 != "warnings"},
                }
        return outs


    @staticmethod
    def _test_logits(data, b: _Batch, W: torch.Tensor) -> List[torch.Tensor]:
        """Held-out logits of every fit: one GEMM per split over that split's test rows
        only (row-chunked), never the full [n, M] product."""
        d = data.d
        bias = W[d] * b.icpt_col
        by_split: Dict[int, List[int]] = {}
        for f in range(b.F):
            by_split.setdefault(b.split_l[f], []).append(f)
        out: List[torch.Tensor] = [None] * b.F
        if getattr(b, "streamed", False):   # one pass over the host rows for every split
            from ..search.cv import ROLE_TEST

            cols_of = {s: torch.cat([torch.arange(b.col0_l[f], b.col0_l[f] + b.K_l[f]) for f in fits]).to(W.device)
                       for s, fits in by_split.items()}
            parts: Dict[int, List[torch.Tensor]] = {s: [] for s in by_split}
            for r0, r1, Xc in data.stream_rows(_lr_stream_chunk(data, b.M)):
                for s_, cols in cols_of.items():
                    m = data.roles[s_, r0:r1] == ROLE_TEST
                    if bool(m.any()):
                        parts[s_].append(torch.addmm(bias[cols], Xc[m], W[:d, cols]))
            for s_, fits in by_split.items():
                Z = torch.cat(parts[s_]) if parts[s_] else torch.empty((0, len(cols_of[s_])), dtype=W.dtype,
                                                                       device=W.device)
                o = 0
                for f in fits:
                    out[f] = Z[:, o:o + b.K_l[f]]
                    o += b.K_l[f]
            return out
        for s, fits in by_split.items():
            te = data.test_rows[s].long()
            cols = torch.cat([torch.arange(b.col0_l[f], b.col0_l[f] + b.K_l[f]) for f in fits]).to(W.device)
            Wc, bc = W[:d, cols], bias[cols]
            step = max(1024, int(2e9 // (4 * (d + len(cols)))))
            Z = torch.cat([torch.addmm(bc, data.X[te[i:i + step]], Wc) for i in range(0, len(te), step)]) \
                if len(te) else torch.empty((0, len(cols)), dtype=W.dtype, device=W.device)
            o = 0
            for f in fits:
                out[f] = Z[:, o:o + b.K_l[f]]
                o += b.K_l[f]
        return out

    def _run_host_lbfgs(self, data, tasks: List[FitTask], keep_models: bool) -> List[FitOutput]:
        from scipy import optimize

        t0 = time.perf_counter()
        X = data.X.detach().double().cpu().numpy()
        y = data.y_cls.cpu().numpy().astype(np.int64)
        C_cls = data.n_classes
        outs = []
        for t in tasks:
            rp = t.params
            tr = data.train_rows[t.split].long().cpu().numpy()
            te = data.test_rows[t.split].long().cpu().numpy()
            Xt, yt = X[tr], y[tr]
            n, d = Xt.shape
            fi = rp["fit_intercept"]
            cwv = class_weight_vector(data, t.split, rp.get("class_weight"))
            sw = np.ones(n) if cwv is None else cwv.cpu().numpy()[yt]
            sw_sum = float(sw.sum())
            lam = 0.0 if rp["C"] is None else 1.0 / (rp["C"] * sw_sum)
            K = 1 if C_cls == 2 else C_cls
            if K == 1:
                tgt = (yt == 1).astype(np.float64)
            else:
                tgt = np.eye(K)[yt]

            def fun(w):
                W = w.reshape((K, d + int(fi)), order="F") if K > 1 else w.reshape(1, -1)
                coef = W[:, :d]
                Z = Xt @ coef.T + (W[:, d] if fi else 0.0)
                if K == 1:
                    z = Z[:, 0]
                    loss = np.sum(sw * (np.logaddexp(0, z) - tgt * z)) / sw_sum
                    r = (sw * (1.0 / (1.0 + np.exp(-z)) - tgt))[:, None] / sw_sum
                else:
                    m = Z.max(1, keepdims=True)
                    lse = m[:, 0] + np.log(np.exp(Z - m).sum(1))
                    loss = np.sum(sw * (lse - (Z * tgt).sum(1))) / sw_sum
                    r = sw[:, None] * (np.exp(Z - lse[:, None]) - tgt) / sw_sum
                loss += 0.5 * lam * np.sum(coef * coef)
                G = np.empty_like(W)
                G[:, :d] = r.T @ Xt + lam * coef
                if fi:
                    G[:, d] = r.sum(0)
                return loss, (G.ravel(order="F") if K > 1 else G.ravel())

            w0 = np.zeros(K * (d + int(fi)))
            res = optimize.minimize(fun, w0, method="L-BFGS-B", jac=True,
                                    options={"maxiter": rp["max_iter"], "maxls": 50, "gtol": rp["tol"],
                                             "ftol": 64 * np.finfo(float).eps})
            W = res.x.reshape((K, d + int(fi)), order="F") if K > 1 else res.x.reshape(1, -1)
            coef, b = W[:, :d], (W[:, d] if fi else np.zeros(K))
            Z = X[te] @ coef.T + b
            if K == 1:
                pred = (Z[:, 0] > 0).astype(np.int32)
                p1 = 1.0 / (1.0 + np.exp(-Z[:, 0]))
                proba = np.stack([1 - p1, p1], 1)
            else:
                pred = Z.argmax(1).astype(np.int32)
                e = np.exp(Z - Z.max(1, keepdims=True))
                proba = e / e.sum(1, keepdims=True)
            warn = list(rp.get("warnings", []))
            if res.status != 0 and res.nit >= rp["max_iter"]:
                warn.append("lbfgs failed to converge (status=1): STOP: TOTAL NO. OF ITERATIONS REACHED LIMIT.")
            o = FitOutput(task_id=t.task_id, pred=torch.from_numpy(pred).to(data.device),
                          proba=torch.from_numpy(proba).to(data.device),
                          info={"warnings": warn, "n_iter": int(res.nit), "host_lbfgs": True})
            if keep_models:
                o.model = {"kind": "linear_logistic", "coef": coef, "intercept": b,
                           "link": KIND_BINARY if K == 1 else KIND_SOFTMAX,
                           "classes": np.asarray(data.classes).tolist(), "model_type": t.model_type,
                           "params": {k2: v for k2, v in rp.items() if k2 != "warnings"}}
            outs.append(o)
        dt = time.perf_counter() - t0
        for o in outs:
            o.fit_seconds = dt / max(1, len(outs))
        return outs


def _ls_solve(A: torch.Tensor, b: torch.Tensor, positive: bool) -> torch.Tensor:
    """Least squares from the normal equations ``A = X^T X``, ``b = X^T y``: the
    minimum-norm solution (sklearn's lstsq), or with ``positive`` the non-negative one
    (sklearn's scipy ``nnls``).  NNLS needs only a factor R with R^T R = A and R^T z = b:
    ||X w - y||^2 = ||R w - z||^2 + const, so the d x d system stands in for the rows."""
    if not positive:
        return torch.linalg.pinv(A, hermitian=True) @ b
    from scipy.optimize import nnls

    lam, V = np.linalg.eigh(A.cpu().numpy())
    keep = lam > lam.max() * A.shape[0] * np.finfo(np.float64).eps if lam.size else lam > 0
    Vk, lk = V[:, keep], lam[keep]
    R = np.sqrt(lk)[:, None] * Vk.T                      # k x d, R^T R = A on its range
    z = (Vk.T @ b.cpu().numpy()) / np.sqrt(lk)           # R^T z = b
    w, _ = nnls(R, z, maxiter=50 * max(1, A.shape[0]))
    return torch.from_numpy(w).to(device=A.device, dtype=torch.float64)


HOST_LBFGS_MAX_WORK = 200_000   # n_train * (d+1) * (K-1): below this a fit runs on the host

_LIN_DEFAULTS = {"fit_intercept": True, "copy_X": True, "n_jobs": None, "positive": False}


def _stream_chunk(data) -> int:
    # float64 working copies of a chunk stay <= ~512 MB whatever d is
    return max(1024, min(data._chunk_rows, (1 << 29) // (8 * (data.d + 2))))


def _lr_stream_chunk(data, M: int) -> int:
    """Rows per streamed chunk of the logistic objective: the chunk's logits and link
    gradient ([rows, M] float32 each) stay <= ~256 MB."""
    return max(1024, min(data._chunk_rows, (1 << 26) // max(1, data.d + 2 * M)))


def streamed_split_moments(data, splits: List[int]) -> Tuple[torch.Tensor, torch.Tensor]:
    """``LinearRegressionFamily.split_moments`` for a table whose float32 rows are not
    resident (DeviceData binned-only): one pass over the host rows in chunks, every split's
    train-row moments of z = [x - c, 1, y - c_y] accumulated in float64 on the device.  The
    shift c is the first chunk's column mean (moments about any shift are exact sums; a shift
    near the mean keeps the centring well conditioned)."""
    from ..search.cv import ROLE_TRAIN

    d = data.d
    dev = data.device
    y = data.y_reg.double()
    S = len(splits)
    M = torch.zeros((S, d + 2, d + 2), dtype=torch.float64, device=dev)
    shift = None
    roles = data.roles[torch.tensor(splits, dtype=torch.long, device=dev)]
    for r0, r1, Xc in data.stream_rows(_stream_chunk(data)):
        Xc = Xc.double()
        yc = y[r0:r1]
        if shift is None:
            shift = torch.cat([Xc.mean(0), yc.mean().view(1)])
        Z = torch.cat([Xc - shift[:d], torch.ones((r1 - r0, 1), dtype=torch.float64, device=dev),
                       (yc - shift[d]).view(-1, 1)], 1)
        for i in range(S):
            Zs = Z[roles[i, r0:r1] == ROLE_TRAIN]
            M[i] += Zs.t() @ Zs
    if shift is None:
        shift = torch.zeros(d + 1, dtype=torch.float64, device=dev)
    return M, shift


def streamed_test_rows(data, split: int, fn):
    """fn(X test rows of the chunk as float64) for every chunk of a binned-only table, the
    results concatenated in test-row order (``data.test_rows[split]`` is ascending)."""
    return streamed_test_many(data, [(split, fn)])[0]


def streamed_test_many(data, jobs):
    """``streamed_test_rows`` for many (split, fn) jobs in ONE pass over the host rows (a
    grid's tasks share the pass instead of re-streaming the table once per task)."""
    from ..search.cv import ROLE_TEST

    parts = [[] for _ in jobs]
    splits = sorted({sp for sp, _ in jobs})
    for r0, r1, Xc in data.stream_rows(_stream_chunk(data)):
        Xd = None
        masks = {}
        for sp in splits:
            m = data.roles[sp, r0:r1] == ROLE_TEST
            if bool(m.any()):
                masks[sp] = m
        if not masks:
            continue
        Xd = Xc.double()
        rows = {sp: Xd[m] for sp, m in masks.items()}
        for i, (sp, fn) in enumerate(jobs):
            if sp in rows:
                parts[i].append(fn(rows[sp]))
    return [torch.cat(p) if p else None for p in parts]


class LinearRegressionFamily(Family):
    model_types = ("LinearRegression",)
    classifiers = ()
    data_parallel = True   # normal-equation moments all-reduced under a RowShard
    streams_rows = True    # binned-only tables: moments and predictions over streamed host rows

    def resolve(self, model_type, params, n_train, n_features, n_classes):
        p = dict(_LIN_DEFAULTS)
        p.update({k: v for k, v in params.items() if k in _LIN_DEFAULTS})
        return {"fit_intercept": as_bool(p["fit_intercept"], "fit_intercept"),
                "positive": as_bool(p["positive"], "positive"), "warnings": []}

    def cost(self, model_type, rp, n_train, n_features, n_classes) -> float:
        return n_train * n_features * n_features * 2e-12 + 1e-3

    def run(self, data, tasks, keep_models=False):
        t0 = time.perf_counter()
        X, y = data.X, data.y_reg
        cache: Dict[tuple, tuple] = {}
        streamed = X is None and getattr(data, "can_stream_rows", lambda: False)()
        if streamed:
            splits = sorted({t.split for t in tasks})
            cache = self._solve_from_moments(data, tasks, streamed_split_moments(data, splits))
        elif (data.is_gpu and not getattr(data, "is_row_shard", False)
                and os.environ.get("DML_LINREG_KERNEL", "1") != "0"):
            cache = self._solve_from_moments(data, tasks)
        outs = []
        preds: Dict[int, torch.Tensor] = {}
        if streamed:   # every task's test predictions from one more pass over the host rows
            keys = [(t.split, t.params["fit_intercept"], bool(t.params.get("positive", False))) for t in tasks]
            uniq = sorted(set(keys), key=keys.index)
            res = streamed_test_many(data, [(k[0], lambda Xt, w=cache[k][0], b0=cache[k][1]: (Xt @ w + b0).float())
                                            for k in uniq])
            byk = dict(zip(uniq, res))
            preds = {i: byk[k] for i, k in enumerate(keys)}
        for ti, t in enumerate(tasks):
            pos = bool(t.params.get("positive", False))
            key = (t.split, t.params["fit_intercept"], pos)
            if key not in cache:
                tr = data.train_rows[t.split].long()
                Xt, yt = X[tr].double(), y[tr].double()
                if getattr(data, "is_row_shard", False):
                    cache[key] = self._sharded_solve(data, Xt, yt, t.params["fit_intercept"], pos)
                elif t.params["fit_intercept"]:
                    xm, ym = Xt.mean(0), yt.mean()
                    Xc, yc = Xt - xm, yt - ym
                else:
                    xm = torch.zeros(data.d, dtype=torch.float64, device=X.device)
                    ym = torch.zeros((), dtype=torch.float64, device=X.device)
                    Xc, yc = Xt, yt
                if key not in cache:
                    w = _ls_solve(Xc.t() @ Xc, Xc.t() @ yc, pos)
                    b0 = ym - xm @ w
                    cache[key] = (w, b0)
            w, b0 = cache[key]
            if streamed:
                pred = preds[ti]
                if pred is None:
                    pred = torch.zeros(0, dtype=torch.float32, device=data.device)
            else:
                te = data.test_rows[t.split].long()
                pred = (X[te].double() @ w + b0).float()
            o = FitOutput(task_id=t.task_id, pred=pred, info={"warnings": t.params.get("warnings", [])})
            if keep_models:
                o.model = {"kind": "linear_regression", "coef": w.cpu().numpy(), "intercept": float(b0),
                           "model_type": t.model_type, "params": {"fit_intercept": t.params["fit_intercept"],
                                                                  "positive": pos}}
            outs.append(o)
        if data.is_gpu:
            torch.cuda.synchronize(data.device)
        dt = time.perf_counter() - t0
        for o in outs:
            o.fit_seconds = dt / max(1, len(outs))
        return outs

    @staticmethod
    def split_moments(data, splits: List[int]) -> Tuple[torch.Tensor, torch.Tensor]:
        """(M [len(splits), d+2, d+2] float64, shift [d+1]): every split's train-row moments
        of z = [x - c_x, 1, y - c_y] from ONE pass over X (csrc/kernels/linear.hip
        ``dml_split_moments``, f64 MFMA), c = the column means over all rows."""
        X = data.X.contiguous()
        y = data.y_reg.float().contiguous() if getattr(data, "y_reg", None) is not None else None
        n, d = X.shape
        dev = X.device
        ymean = torch.mean(y, dtype=torch.float64).view(1) if y is not None else torch.zeros(1, dtype=torch.float64,
                                                                                               device=dev)
        shift = torch.cat([torch.mean(X, 0, dtype=torch.float64), ymean])
        Dp = _roundup(d + 2, 16)
        roles = data.roles[torch.tensor(splits, dtype=torch.long, device=dev)].contiguous()
        out = torch.zeros((len(splits), Dp, Dp), dtype=torch.float64, device=dev)
        lib = native.hip_lib()
        for g0 in range(0, len(splits), 8):
            g1 = min(len(splits), g0 + 8)
            rc = lib.dml_split_moments(native.ptr(X), X.stride(0), native.ptr(y), native.ptr(shift),
                                       native.ptr(roles[g0:g1]), n, d, g1 - g0, native.ptr(out[g0:g1]), Dp,
                                       native.stream_handle(dev))
            if rc:
                raise RuntimeError(f"dml_split_moments failed ({rc})")
        M = torch.triu(out) + torch.triu(out, 1).transpose(1, 2)   # the kernel fills ti <= tj tiles
        return M[:, :d + 2, :d + 2], shift

    def _solve_from_moments(self, data, tasks, moments=None) -> Dict[tuple, tuple]:
        """(split, fit_intercept) -> (w, b0) for every task, from the fused moments
        (``moments``: precomputed (M, shift), e.g. streamed from host rows)."""
        d = data.d
        splits = sorted({t.split for t in tasks})
        M, shift = moments if moments is not None else self.split_moments(data, splits)
        cx, cy = shift[:d], shift[d]
        out: Dict[tuple, tuple] = {}
        for i, sp in enumerate(splits):
            m = M[i]
            cnt, Sx, Sy = m[d, d], m[:d, d], m[d + 1, d]
            XX, Xy = m[:d, :d], m[:d, d + 1]
            for fi, pos in sorted({(t.params["fit_intercept"], bool(t.params.get("positive", False)))
                                   for t in tasks if t.split == sp}):
                if fi:
                    xm, ym = Sx / cnt.clamp_min(1), Sy / cnt.clamp_min(1)
                    A = XX - cnt * torch.outer(xm, xm)
                    b = Xy - cnt * xm * ym
                    w = _ls_solve(A, b, pos)
                    out[(sp, fi, pos)] = (w, (ym + cy) - (xm + cx) @ w)
                else:   # moments about the origin: x = z + c_x, y = z_y + c_y
                    XX0 = XX + torch.outer(Sx, cx) + torch.outer(cx, Sx) + cnt * torch.outer(cx, cx)
                    Xy0 = Xy + Sx * cy + cx * Sy + cnt * cx * cy
                    w = _ls_solve(XX0, Xy0, pos)
                    out[(sp, fi, pos)] = (w, torch.zeros((), dtype=torch.float64, device=w.device))
        return out

    @staticmethod
    def _sharded_solve(data, Xt: torch.Tensor, yt: torch.Tensor, fit_intercept: bool, positive: bool = False):
        """Normal equations from all-reduced shard moments: one all-reduce of
        [count, sum x, sum y, X^T X, X^T y] (float64), centred on the global means."""
        d = Xt.shape[1]
        m = torch.cat([torch.tensor([float(Xt.shape[0])], dtype=torch.float64, device=Xt.device), Xt.sum(0),
                       yt.sum().view(1), (Xt.t() @ Xt).flatten(), Xt.t() @ yt])
        _dp_sum(data, m)
        cnt, sx, sy = m[0], m[1:1 + d], m[1 + d]
        XX = m[2 + d:2 + d + d * d].view(d, d)
        Xy = m[2 + d + d * d:]
        if fit_intercept:
            xm, ym = sx / cnt.clamp_min(1), sy / cnt.clamp_min(1)
            A = XX - cnt * torch.outer(xm, xm)
            bvec = Xy - cnt * xm * ym
        else:
            xm = torch.zeros(d, dtype=torch.float64, device=Xt.device)
            ym = torch.zeros((), dtype=torch.float64, device=Xt.device)
            A, bvec = XX, Xy
        w = _ls_solve(A, bvec, positive)
        return w, ym - xm @ w


register(LogisticFamily())
register(LinearRegressionFamily())
