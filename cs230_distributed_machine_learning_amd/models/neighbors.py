"""KNeighborsClassifier / KNeighborsRegressor — one neighbour search per job, not per fit.

Reference: both are whitelisted (aws-prod/worker/worker.py:42,49) and sklearn fits /
predicts them once per (candidate, fold): a KD/ball tree build plus a query pass each
time (sklearn ``neighbors/_kd_tree``, ``_ball_tree``, ``_pairwise_distances_reduction``).

Here a KNN "fit" is only the choice of training rows (a role row of the split tensor),
so for every metric the job uses ONE exact brute-force pass (HIP kernel ``dml_knn``,
csrc/kernels/neighbors.hip; torch on CPU) finds the ``K_max`` nearest training rows of
every test row of every split; each candidate (n_neighbors, weights) then votes from a
prefix of those lists.  Neighbour search is exact, so predictions match sklearn's
brute/kd/ball algorithms except where equal distances make the k-th neighbour
ambiguous (ties resolved by lower row index here; parity unpinned for exact ties).
``metric="cosine"`` is a library GEMM over unit rows (sklearn's cosine_distances).
``algorithm`` / ``leaf_size`` only pick sklearn's search structure and are accepted
and ignored.
"""
from __future__ import annotations

import math
import os
import time
from typing import Any, Dict, List, Tuple

import numpy as np
import torch

from ..utils import native
from .base import Family, FitOutput, FitTask, ParamError, as_int, as_float, register

_DEFAULTS = {"n_neighbors": 5, "weights": "uniform", "algorithm": "auto", "leaf_size": 30, "p": 2,
             "metric": "minkowski", "metric_params": None, "n_jobs": None}
M_L2, M_L1, M_LINF, M_P, M_COS = 0, 1, 2, 3, 4
KERNEL_KMAX = 64

_METRICS = {"euclidean": (M_L2, 2.0), "l2": (M_L2, 2.0), "manhattan": (M_L1, 1.0), "cityblock": (M_L1, 1.0),
            "l1": (M_L1, 1.0), "chebyshev": (M_LINF, math.inf), "infinity": (M_LINF, math.inf),
            "cosine": (M_COS, 0.0)}


def metric_code(metric: str, p) -> Tuple[int, float]:
    metric = str(metric).lower()
    if metric == "minkowski":
        p = as_float(p, "p", lo=0.0)
        if p < 1:
            raise ParamError("p must be >= 1 for the minkowski metric")
        if p == 1:
            return M_L1, 1.0
        if p == 2:
            return M_L2, 2.0
        if math.isinf(p):
            return M_LINF, math.inf
        return M_P, p
    if metric in _METRICS:
        return _METRICS[metric]
    raise ParamError(f"metric {metric!r} is not supported (minkowski/euclidean/manhattan/chebyshev/cosine)")


def finish_distance(acc: torch.Tensor, metric: int, p: float) -> torch.Tensor:
    """Kernel accumulators -> true distances (sqrt / p-th root)."""
    if metric == M_L2:
        return acc.clamp_min(0).sqrt()
    if metric == M_P:
        return acc.clamp_min(0).pow(1.0 / p)
    return acc


def _unit_rows(A: torch.Tensor) -> torch.Tensor:
    n = torch.linalg.vector_norm(A, dim=1, keepdim=True)
    return A / torch.where(n > 0, n, torch.ones_like(n))     # zero rows stay zero (sklearn normalize)


def _acc_torch(Q: torch.Tensor, R: torch.Tensor, metric: int, p: float) -> torch.Tensor:
    """Accumulator-space distances [q, r] (same quantity the kernel ranks by)."""
    if metric == M_COS:   # sklearn cosine_distances: clip(1 - <q/|q|, r/|r|>, 0, 2); a library GEMM
        return (1.0 - _unit_rows(Q) @ _unit_rows(R).t()).clamp(0.0, 2.0)
    diff = (Q[:, None, :] - R[None, :, :]).abs()
    if metric == M_L2:
        return (diff * diff).sum(2)
    if metric == M_L1:
        return diff.sum(2)
    if metric == M_LINF:
        return diff.amax(2)
    return diff.pow(p).sum(2)


def knn_search_torch(X: torch.Tensor, qrows: torch.Tensor, train_rows: torch.Tensor, K: int, metric: int, p: float):
    """(acc distances [q, K], global row ids [q, K]) — ties broken by lower row id."""
    out_d, out_i = [], []
    R = X[train_rows.long()]
    nr = R.shape[0]
    K = min(K, nr)
    step = max(1, (1 << 24) // max(1, nr * max(1, X.shape[1] // 8)))
    for s in range(0, qrows.numel(), step):
        Q = X[qrows[s:s + step].long()]
        D = _acc_torch(Q, R, metric, p)
        # stable sort over ascending row ids == (distance, row) order
        Ds, idx = torch.sort(D, dim=1, stable=True)
        out_d.append(Ds[:, :K])
        out_i.append(train_rows.long()[idx[:, :K]])
    if not out_d:
        return (torch.empty((0, K), dtype=X.dtype, device=X.device),
                torch.empty((0, K), dtype=torch.long, device=X.device))
    return torch.cat(out_d), torch.cat(out_i)


MFMA_KMAX = 32   # the matrix-core path re-ranks 64 candidates: keep >= 32 rows of margin


def mfma_operands(data):
    """bf16 hi/lo planes of X in the MFMA K-step layout [2][KS][npad][16] plus the squared
    row norms (csrc/kernels/neighbors.hip ``dml_knn_l2_mfma``); built once per dataset."""
    ops = getattr(data, "_knn_mfma_ops", None)
    if ops is None:
        X = data.X
        n, d = X.shape
        ks = -(-d // 16)
        if ks <= 8:
            ks = 1 << (ks - 1).bit_length()   # register-resident query operand: 1/2/4/8 K-steps
        npad = -(-n // 128) * 128
        Xp = torch.zeros((npad, ks * 16), dtype=torch.float32, device=X.device)
        Xp[:n, :d] = X
        hi = Xp.to(torch.bfloat16)
        lo = (Xp - hi.float()).to(torch.bfloat16)
        xhl = torch.stack([hi, lo]).view(2, npad, ks, 16).transpose(1, 2).contiguous()
        rn = (X.double() ** 2).sum(1).float().contiguous()
        ops = (xhl, npad, ks, rn)
        data._knn_mfma_ops = ops
    return ops


def knn_search_hip(data, splits: List[int], K: int, metric: int, p: float) -> Dict[int, Tuple[torch.Tensor, torch.Tensor]]:
    """One kernel launch for all test rows of all ``splits``: squared L2 with K <= 32 on the
    matrix cores (exact re-rank of an MFMA-selected top-64), every other metric on the
    scalar streaming kernel."""
    lib = native.hip_lib()
    qpw = int(lib.dml_knn_qpw())
    dev = data.device
    use_mfma = metric == M_L2 and K <= MFMA_KMAX and os.environ.get("DML_KNN_MFMA", "1") != "0"
    qr, qs, spans = [], [], {}
    off = 0
    for s in splits:
        rows = data.test_rows[s].long()
        m = rows.numel()
        pad = (-m) % qpw
        qr.append(torch.cat([rows, torch.full((pad,), -1, dtype=torch.long, device=dev)]))
        qs.append(torch.full((m + pad,), s, dtype=torch.long, device=dev))
        spans[s] = (off, m)
        off += m + pad
    if use_mfma:   # whole workgroups of 4 query groups
        pad = (-off) % (4 * qpw)
        qr.append(torch.full((pad,), -1, dtype=torch.long, device=dev))
        qs.append(torch.full((pad,), splits[-1], dtype=torch.long, device=dev))
    qrow = torch.cat(qr).to(torch.int32).contiguous()
    qsplit = torch.cat(qs).to(torch.int32).contiguous()
    groups = qrow.numel() // qpw
    out_d = torch.empty((qrow.numel(), K), dtype=torch.float32, device=dev)
    out_i = torch.empty((qrow.numel(), K), dtype=torch.int32, device=dev)
    if use_mfma:
        xhl, npad, ks, rn = mfma_operands(data)
        rc = lib.dml_knn_l2_mfma(native.ptr(xhl), npad, ks, native.ptr(rn), native.ptr(data.X), data.n, data.d,
                                 native.ptr(data.roles), native.ptr(qrow), native.ptr(qsplit), groups, K,
                                 native.ptr(out_d), native.ptr(out_i), native.stream_handle(dev))
    else:
        XT = data.feature_major()
        rc = lib.dml_knn(native.ptr(data.X), native.ptr(XT), data.n, data.d, native.ptr(data.roles), native.ptr(qrow),
                         native.ptr(qsplit), groups, metric, float(p if math.isfinite(p) else 0.0), K,
                         native.ptr(out_d), native.ptr(out_i), native.stream_handle(dev))
    if rc:
        raise RuntimeError(f"dml_knn failed (rc={rc})")
    return {s: (out_d[o:o + m], out_i[o:o + m].long()) for s, (o, m) in spans.items()}


def vote(dist: torch.Tensor, nb_y: torch.Tensor, k: int, weights: str, n_classes: int, classification: bool):
    """Prediction from the first ``k`` neighbours (sklearn's uniform / distance rules)."""
    d = dist[:, :k].double()
    y = nb_y[:, :k]
    if weights == "distance":
        w = 1.0 / d                                      # 0-distance -> inf
        inf = torch.isinf(w)
        row_inf = inf.any(1, keepdim=True)
        w = torch.where(row_inf, inf.double(), w)
    else:
        w = torch.ones_like(d)
    if classification:
        scores = torch.zeros((d.shape[0], n_classes), dtype=torch.float64, device=d.device)
        scores.scatter_add_(1, y.long(), w)
        pred = scores.argmax(1).to(torch.int32)          # first max = smallest class (sklearn mode)
        proba = scores / scores.sum(1, keepdim=True).clamp_min(1e-300)
        return pred, proba
    yv = y.double()
    return ((w * yv).sum(1) / w.sum(1)).float(), None


def _merge_topk(d_parts: torch.Tensor, i_parts: torch.Tensor, y_parts: torch.Tensor, K: int, with_ids: bool = False):
    """[W, q, K] per-rank candidates -> the global top-K per query in (distance, row id)
    order: the order a one-process stable sort over ascending row ids gives."""
    W, q, k = d_parts.shape
    d = d_parts.permute(1, 0, 2).reshape(q, W * k)
    i = i_parts.permute(1, 0, 2).reshape(q, W * k)
    y = y_parts.permute(1, 0, 2).reshape(q, W * k)
    _, o1 = torch.sort(i, dim=1, stable=True)                  # ascending row id ...
    d, i, y = d.gather(1, o1), i.gather(1, o1), y.gather(1, o1)
    _, o2 = torch.sort(d, dim=1, stable=True)                  # ... then distance (stable)
    if with_ids:
        return d.gather(1, o2)[:, :K], i.gather(1, o2)[:, :K], y.gather(1, o2)[:, :K]
    return d.gather(1, o2)[:, :K], y.gather(1, o2)[:, :K]


class _QueryTable:
    """This rank's rows followed by the gathered held-out rows of every split, as one table
    for ``knn_search_hip``: candidates are this rank's training rows (role 1), queries are
    the appended rows (role 0), so the HIP kernels search other ranks' queries unchanged."""

    def __init__(self, data, Qs: Dict[int, torch.Tensor]):
        self.device, self.d, n = data.device, data.d, data.n
        self.X = torch.cat([data.X] + [Qs[s] for s in sorted(Qs)]).contiguous()
        self.n = int(self.X.shape[0])
        self.roles = torch.zeros((data.roles.shape[0], self.n), dtype=torch.uint8, device=self.device)
        self.roles[:, :n] = data.roles
        self.test_rows, off = {}, n
        for s in sorted(Qs):
            m = int(Qs[s].shape[0])
            self.test_rows[s] = torch.arange(off, off + m, dtype=torch.int32, device=self.device)
            off += m

    def feature_major(self) -> torch.Tensor:
        if getattr(self, "_XT", None) is None:
            self._XT = self.X.t().contiguous()
        return self._XT


def knn_search_sharded(data, splits: List[int], K: int, metric: int, p: float, y: torch.Tensor):
    """Row-sharded search (parallel/data_parallel.py RowShard): every rank searches ALL
    of a split's held-out rows (one all-gather of their features) against its OWN training
    rows, one all-gather of the per-rank top-K (distance, global row id, target) and an
    exact merge give the global neighbours; each rank keeps its own queries' rows.
    Distances are computed element for element like the one-process search, so ties break
    the same way (lower global row id)."""
    out = {}
    world, rank = data.world, data.rank
    Qs = {s: data._gather_rows(data.X[data.test_rows[s].long()], data._test_counts[s]) for s in splits}
    hip = None
    # the HIP search (MFMA for L2) needs K candidates on this rank for every split
    if (data.is_gpu and K <= KERNEL_KMAX and metric != M_COS
            and all(int(data.train_rows[s].numel()) >= K for s in splits)):
        hip = knn_search_hip(_QueryTable(data, Qs), splits, K, metric, p)
    for s in splits:
        cnt = data._test_counts[s]
        Q = Qs[s]                                                              # [m_glob, d]
        tr = data.train_rows[s].long()
        R = data.X[tr]
        m = Q.shape[0]
        k_loc = min(K, R.shape[0])
        big = torch.finfo(torch.float32).max
        dd = torch.full((m, K), big, dtype=torch.float32, device=Q.device)
        ii = torch.full((m, K), 2 ** 62, dtype=torch.long, device=Q.device)
        yy = torch.zeros((m, K), dtype=y.dtype, device=Q.device)
        if hip is not None:   # indices < data.n: this rank's rows
            acc, idx = hip[s]
            dd, ii, yy = acc.float(), idx + data.r0, y[idx]
        elif k_loc > 0 and m > 0:
            step = max(1, (1 << 24) // max(1, R.shape[0] * max(1, data.d // 8)))
            for q0 in range(0, m, step):
                D = _acc_torch(Q[q0:q0 + step], R, metric, p)
                Ds, idx = torch.sort(D, dim=1, stable=True)
                dd[q0:q0 + step, :k_loc] = Ds[:, :k_loc].float()
                ii[q0:q0 + step, :k_loc] = tr[idx[:, :k_loc]] + data.r0
                yy[q0:q0 + step, :k_loc] = y[tr[idx[:, :k_loc]]]
        acc, nb_y = _merge_topk(data.all_gather_equal(dd).view(world, m, K),
                                data.all_gather_equal(ii).view(world, m, K),
                                data.all_gather_equal(yy).view(world, m, K), K)
        o = int(cnt[:rank].sum())
        out[s] = (acc[o:o + int(cnt[rank])], nb_y[o:o + int(cnt[rank])])
    return out


class _ChunkTable:
    """One streamed chunk of training candidates [r0, r1) followed by a block of query rows,
    as a table for ``knn_search_hip`` (the role rows of the chunk's rows; queries role 0)."""

    def __init__(self, data, r0: int, Xc: torch.Tensor, Q: torch.Tensor, qpos: Dict[int, Tuple[int, int]]):
        self.device, self.d = data.device, data.d
        nc = int(Xc.shape[0])
        self.X = torch.cat([Xc, Q]).contiguous()
        self.n = int(self.X.shape[0])
        self.roles = torch.zeros((data.roles.shape[0], self.n), dtype=torch.uint8, device=self.device)
        self.roles[:, :nc] = data.roles[:, r0:r0 + nc]
        self.test_rows = {s: torch.arange(nc + a, nc + b, dtype=torch.int32, device=self.device)
                          for s, (a, b) in qpos.items()}

    def feature_major(self) -> torch.Tensor:
        if getattr(self, "_XT", None) is None:
            self._XT = self.X.t().contiguous()
        return self._XT


def knn_search_streamed(data, splits: List[int], K: int, metric: int, p: float, y: torch.Tensor):
    """Binned-only tables (float32 rows too large for HBM, DeviceData.stream_rows): the
    queries -- every split's held-out rows -- are taken in blocks that fit a device budget
    (``DML_KNN_QBLOCK_GB``, default 8); per block the host rows stream past once in chunks,
    each chunk's training rows are searched exactly (HIP kernels as for a resident table, or
    torch) and merged into the running top-K in (distance, row id) order -- the order of the
    one-pass search, so the neighbours equal the resident path's."""
    Xh = data._X_host
    dev = data.device
    budget = float(os.environ.get("DML_KNN_QBLOCK_GB", "8")) * 1e9
    per_block = max(1, int(budget // max(1, 4 * data.d)))
    big = torch.finfo(torch.float32).max
    # (split, [a, b)) slices of each split's ascending test rows, grouped into query blocks
    work, cur, used = [], [], 0
    for s in splits:
        rows = data.test_rows[s].long()
        for a in range(0, rows.numel(), per_block):
            b = min(rows.numel(), a + per_block)
            if used + (b - a) > per_block and cur:
                work.append(cur)
                cur, used = [], 0
            cur.append((s, a, b))
            used += b - a
    if cur:
        work.append(cur)
    res = {s: ([], []) for s in splits}
    for block in work:
        qidx = torch.cat([data.test_rows[s].long()[a:b] for s, a, b in block])
        Q = torch.from_numpy(np.array(Xh[qidx.cpu().numpy()], dtype=np.float32)).to(dev)
        qpos, off = {}, 0
        for s, a, b in block:
            qpos[s] = (off, off + (b - a))
            off += b - a
        m = off
        dd = torch.full((m, K), big, dtype=torch.float32, device=dev)
        ii = torch.full((m, K), 2 ** 62, dtype=torch.long, device=dev)
        yy = torch.zeros((m, K), dtype=y.dtype, device=dev)
        for r0, r1, Xc in data.stream_rows():
            tab = _ChunkTable(data, r0, Xc, Q, qpos)
            enough = all(int((tab.roles[s, :r1 - r0] == 1).sum()) >= K for s in qpos)
            if data.is_gpu and K <= KERNEL_KMAX and metric != M_COS and enough:
                got = knn_search_hip(tab, sorted(qpos), K, metric, p)
                cd = torch.cat([got[s][0].float() for s, _, _ in block])
                ci = torch.cat([got[s][1] for s, _, _ in block]) + r0
            else:
                cd = torch.full((m, K), big, dtype=torch.float32, device=dev)
                ci = torch.full((m, K), 2 ** 62, dtype=torch.long, device=dev)
                for s, (a, b) in qpos.items():
                    tr = torch.nonzero(tab.roles[s, :r1 - r0] == 1).flatten()
                    if tr.numel() == 0:
                        continue
                    acc, idx = knn_search_torch(tab.X, tab.test_rows[s], tr, K, metric, p)
                    k = acc.shape[1]
                    cd[a:b, :k] = acc.float()
                    ci[a:b, :k] = idx + r0
            cy = y[ci.clamp_max(data.n - 1)]
            dd, ii, yy = _merge_topk(torch.stack([dd, cd]), torch.stack([ii, ci]), torch.stack([yy, cy]), K,
                                     with_ids=True)
        for s, (a, b) in qpos.items():
            res[s][0].append(dd[a:b])
            res[s][1].append(yy[a:b])
    return {s: (torch.cat(res[s][0]), torch.cat(res[s][1])) for s in splits}


class KNeighborsFamily(Family):
    model_types = ("KNeighborsClassifier", "KNeighborsRegressor")
    classifiers = ("KNeighborsClassifier",)
    data_parallel = True   # row-sharded search: per-rank top-K + exact merge (knn_search_sharded)
    dp_when_few = False    # a replicated table is always faster when it fits
    streams_rows = True    # binned-only tables: exact search over streamed host chunks

    def resolve(self, model_type, params, n_train, n_features, n_classes):
        p = dict(_DEFAULTS)
        p.update({k: v for k, v in params.items() if k in _DEFAULTS})
        warn = []
        unknown = sorted(k for k in params if k not in _DEFAULTS)
        if unknown:
            warn.append(f"ignored unknown parameters {unknown}")
        k = as_int(p["n_neighbors"], "n_neighbors", lo=1)
        weights = p["weights"] if p["weights"] is not None else "uniform"
        if weights not in ("uniform", "distance"):
            raise ParamError("weights not recognized: should be 'uniform', 'distance'")
        if p["algorithm"] not in ("auto", "ball_tree", "kd_tree", "brute"):
            raise ParamError(f"algorithm {p['algorithm']!r} invalid")
        as_int(p["leaf_size"], "leaf_size", lo=1)
        if p["metric_params"]:
            raise ParamError("metric_params is not supported")
        metric, pp = metric_code(p["metric"], p["p"])
        return {"n_neighbors": k, "weights": weights, "metric": metric, "p": pp, "warnings": warn}

    def cost(self, model_type, rp, n_train, n_features, n_classes) -> float:
        # one search per job is shared by every candidate; price a candidate at a share
        return n_train * max(1.0, n_train / 4) * max(1, n_features) * 2e-13 + 1e-3

    def run(self, data, tasks: List[FitTask], keep_models: bool = False) -> List[FitOutput]:
        if not tasks:
            return []
        t0 = time.perf_counter()
        clf = data.classification
        y = data.y_cls if clf else data.y_reg
        outs: Dict[int, FitOutput] = {}
        groups: Dict[Tuple[int, float], List[FitTask]] = {}
        for t in tasks:
            groups.setdefault((t.params["metric"], t.params["p"]), []).append(t)
        for (metric, p), ts in groups.items():
            splits = sorted({t.split for t in ts})
            for t in ts:
                if t.params["n_neighbors"] > data.train_counts[t.split]:
                    outs[t.task_id] = FitOutput(task_id=t.task_id, error=(
                        f"Expected n_neighbors <= n_samples_fit, but n_neighbors = {t.params['n_neighbors']}, "
                        f"n_samples_fit = {data.train_counts[t.split]}"))
            ok = [t for t in ts if t.task_id not in outs]
            if not ok:
                continue
            kmax = max(t.params["n_neighbors"] for t in ok)
            if getattr(data, "is_row_shard", False):
                nb = knn_search_sharded(data, splits, kmax, metric, p, y)
            elif data.X is None and getattr(data, "can_stream_rows", lambda: False)():
                nb = knn_search_streamed(data, splits, kmax, metric, p, y)
            elif data.is_gpu and kmax <= KERNEL_KMAX and metric != M_COS:
                nb = {s: (a, y[i]) for s, (a, i) in knn_search_hip(data, splits, kmax, metric, p).items()}
            else:
                nb = {s: (a, y[i]) for s, (a, i) in ((s, knn_search_torch(data.X, data.test_rows[s], data.train_rows[s],
                                                                          kmax, metric, p)) for s in splits)}
            for t in ok:
                acc, nb_y = nb[t.split]
                dist = finish_distance(acc, metric, p)
                pred, proba = vote(dist, nb_y, t.params["n_neighbors"], t.params["weights"], data.n_classes, clf)
                o = FitOutput(task_id=t.task_id, pred=pred, proba=proba, info={"warnings": t.params["warnings"]})
                if keep_models:
                    tr = data.train_rows[t.split].long()
                    if data.X is None:   # binned-only: the artefact's training rows from the host table
                        Xtr = torch.from_numpy(np.array(data._X_host[tr.cpu().numpy()], dtype=np.float32))
                    else:
                        Xtr = data.X[tr]
                    ytr = y[tr]
                    if getattr(data, "is_row_shard", False):   # the fitted model holds every rank's rows
                        cnt = data.all_gather_equal(torch.tensor([tr.numel()], device=data.device)).cpu().numpy()
                        Xtr, ytr = data._gather_rows(Xtr, cnt), data._gather_rows(ytr, cnt)
                    o.model = {"kind": "knn", "X": Xtr.cpu().numpy(), "y": ytr.cpu().numpy(),
                               "classes": None if not clf else np.asarray(data.classes).tolist(),
                               "n_neighbors": t.params["n_neighbors"], "weights": t.params["weights"],
                               "metric": metric, "p": p, "model_type": t.model_type, "n_classes": data.n_classes}
                outs[t.task_id] = o
        data.sync()
        dt = time.perf_counter() - t0
        for o in outs.values():
            o.fit_seconds = dt / max(1, len(outs))
        return [outs[t.task_id] for t in tasks]


def knn_predict_numpy(model: Dict[str, Any], X: np.ndarray) -> np.ndarray:
    """Host prediction for a saved KNN artefact (the artefact stores its training rows)."""
    Xtr = torch.from_numpy(np.asarray(model["X"], dtype=np.float32))
    ytr = torch.from_numpy(np.asarray(model["y"]))
    Q = torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32))
    allX = torch.cat([Xtr, Q])
    n = Xtr.shape[0]
    metric, p, k = int(model["metric"]), float(model["p"]), int(model["n_neighbors"])
    acc, idx = knn_search_torch(allX, torch.arange(n, n + Q.shape[0]), torch.arange(n), k, metric, p)
    clf = model.get("classes") is not None
    pred, _ = vote(finish_distance(acc, metric, p), ytr[idx], k, model["weights"], int(model.get("n_classes", 1)), clf)
    pred = pred.numpy()
    return np.asarray(model["classes"])[pred] if clf else pred


register(KNeighborsFamily())
