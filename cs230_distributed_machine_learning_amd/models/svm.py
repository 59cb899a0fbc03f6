"""SVC / SVR — every dual problem of a job solved in one batched SMO launch.

Reference: both are whitelisted (aws-prod/worker/worker.py:40,47); sklearn fits them per
(candidate, fold) with libsvm (``svm/_libsvm``, C++ SMO), one-vs-one for multiclass.

Here each (candidate, split[, class pair]) is one dual problem for the batched solver
(csrc/kernels/svm.hip on the GPU, csrc/runtime/svm_cpu.cpp on the host), which runs
libsvm's algorithm (WSS3 selection, same update / stopping rule / tie rules), so the
support vectors and decision values match libsvm up to float round-off in the kernel
values.  Rows of each (split, class pair) are gathered ONCE into a feature-major block
shared by every candidate using it.  Decision values for held-out rows are kernel
matrix x coefficient products (library GEMM).  Supported: C, kernel
(linear/poly/rbf/sigmoid), degree, gamma ('scale'/'auto'/float), coef0, tol, max_iter,
class_weight (dict / 'balanced'), epsilon (SVR).  ``shrinking`` / ``cache_size`` only
affect libsvm's speed and are accepted and ignored; ``probability=True`` does not change
``predict`` and is ignored (reported); ``break_ties=True`` predicts the argmax of
sklearn's one-vs-rest decision function (votes + squashed summed confidences).
"""
from __future__ import annotations

import ctypes
import math
import os
import time
from typing import Any, Dict, List, Tuple

import numpy as np
import torch

from ..utils import native
from .base import Family, FitOutput, FitTask, ParamError, as_bool, as_float, as_int, register

_SVC = "SVC"
_SVR = "SVR"
KLIN, KPOLY, KRBF, KSIG = 0, 1, 2, 3
_KERNELS = {"linear": KLIN, "poly": KPOLY, "rbf": KRBF, "sigmoid": KSIG}

_SVC_DEFAULTS = {"C": 1.0, "kernel": "rbf", "degree": 3, "gamma": "scale", "coef0": 0.0, "shrinking": True,
                 "probability": False, "tol": 1e-3, "cache_size": 200, "class_weight": None, "verbose": False,
                 "max_iter": -1, "decision_function_shape": "ovr", "break_ties": False, "random_state": None}
_SVR_DEFAULTS = {"kernel": "rbf", "degree": 3, "gamma": "scale", "coef0": 0.0, "tol": 1e-3, "C": 1.0,
                 "epsilon": 0.1, "shrinking": True, "cache_size": 200, "verbose": False, "max_iter": -1}

PROB_DTYPE = np.dtype([("xoff", "<i8"), ("roff", "<i8"), ("nrows", "<i8"), ("L", "<i8"), ("voff", "<i8"),
                       ("koff", "<i8"), ("kernel", "<i8"), ("degree", "<i8"), ("gamma", "<f8"), ("coef0", "<f8"),
                       ("eps", "<f8"), ("max_iter", "<i8"), ("iters", "<i8"), ("status", "<i8"), ("svr", "<i8"),
                       ("coff", "<i8"), ("moff", "<i8")])
CHUNK_ITERS = 20000
SPLIT_CHUNK_ITERS = 50000
CACHE_FRACTION = 0.25        # of free HBM for the kernel-column caches (libsvm cache_size analogue) ...
CACHE_MAX_GB = 48.0          # ... and at most this much (DML_SVM_CACHE_GB; 288 GB of HBM per MI355X)
MIN_ROWS_PER_WG = 1024       # split a problem over workgroups only down to this slice size



def _ovr_argmax(dec, ti, pairs, m, C, dev) -> torch.Tensor:
    """sklearn SVC(break_ties=True): argmax of the one-vs-rest decision function built from
    the one-vs-one values (sklearn.utils.multiclass._ovr_decision_function: votes plus
    summed confidences squashed into (-1/3, 1/3))."""
    votes = torch.zeros((m, C), dtype=torch.float64, device=dev)
    conf = torch.zeros((m, C), dtype=torch.float64, device=dev)
    for pi, (a_, b_) in enumerate(pairs):
        dv = dec.get((ti, pi))
        if dv is None:
            continue
        dv = dv.double()
        conf[:, a_] += dv
        conf[:, b_] -= dv
        votes[:, a_] += (dv >= 0).double()
        votes[:, b_] += (dv < 0).double()
    return (votes + conf / (3 * (conf.abs() + 1))).argmax(1).to(torch.int32)

class SVMFamily(Family):
    model_types = (_SVC, _SVR)
    # binned-only tables (float32 rows too large for HBM): the fits run on the host rows with
    # the host SMO -- the reference trains SVC/SVR on any table that fits in RAM
    # (aws-prod/worker/worker.py:40,47,406-425); engine/executor.py run_candidates
    host_ok = True
    classifiers = (_SVC,)

    def resolve(self, model_type, params, n_train, n_features, n_classes) -> Dict[str, Any]:
        defaults = _SVC_DEFAULTS if model_type == _SVC else _SVR_DEFAULTS
        p = dict(defaults)
        p.update({k: v for k, v in params.items() if k in defaults})
        warn = []
        unknown = sorted(k for k in params if k not in defaults)
        if unknown:
            warn.append(f"ignored unknown parameters {unknown}")
        kernel = p["kernel"]
        if kernel not in _KERNELS:
            raise ParamError(f"kernel {kernel!r} is not supported (linear/poly/rbf/sigmoid)")
        C = as_float(p["C"], "C")
        if C <= 0:
            raise ParamError("C <= 0")
        gamma = p["gamma"]
        if isinstance(gamma, str):
            if gamma not in ("scale", "auto"):
                raise ParamError(f"gamma {gamma!r} invalid")
        else:
            gamma = as_float(gamma, "gamma", lo=0.0)
        out = {"C": C, "kernel": _KERNELS[kernel], "degree": as_int(p["degree"], "degree", lo=0),
               "gamma": gamma, "coef0": as_float(p["coef0"], "coef0"), "tol": as_float(p["tol"], "tol", lo=0.0),
               "max_iter": as_int(p["max_iter"], "max_iter", lo=-1), "warnings": warn}
        if model_type == _SVR:
            out["epsilon"] = as_float(p["epsilon"], "epsilon", lo=0.0)
        else:
            cw = p["class_weight"]
            if cw not in (None, "balanced") and not isinstance(cw, dict):
                raise ParamError("class_weight must be None, 'balanced' or a dict")
            out["class_weight"] = cw
            if as_bool(p["probability"], "probability"):
                warn.append("probability=True: Platt scaling not computed (predict is unaffected)")
            out["break_ties"] = as_bool(p["break_ties"], "break_ties")
            if out["break_ties"] and p["decision_function_shape"] == "ovo":
                raise ParamError("break_ties must be False when decision_function_shape is 'ovo'")
        return out

    def cost(self, model_type, rp, n_train, n_features, n_classes) -> float:
        pairs = n_classes * (n_classes - 1) / 2 if model_type == _SVC and n_classes > 2 else 1
        per = n_train / max(1, pairs) if pairs > 1 else n_train
        return pairs * per * per * max(1, n_features) * 2e-11 + 1e-2

    # ------------------------------------------------------------------------------------
    def run(self, data, tasks: List[FitTask], keep_models: bool = False) -> List[FitOutput]:
        if not tasks:
            return []
        t0 = time.perf_counter()
        dev = data.device
        svr = not data.classification
        C_cls = data.n_classes
        pairs = [(None, None)] if svr else [(a, b) for a in range(C_cls) for b in range(a + 1, C_cls)]
        # ---- rowsets (split, pair) shared by candidates ----------------------------------
        rowsets: Dict[Tuple[int, Any], torch.Tensor] = {}
        for t in tasks:
            tr = data.train_rows[t.split].long()
            for pr in pairs:
                key = (t.split, pr)
                if key in rowsets:
                    continue
                if svr:
                    rowsets[key] = tr
                else:
                    yt = data.y_cls[tr]
                    rowsets[key] = tr[(yt == pr[0]) | (yt == pr[1])]
        keys = list(rowsets)
        xoff, off = {}, 0
        blocks = []
        for k in keys:
            r = rowsets[k]
            blocks.append(data.X[r].t().contiguous().reshape(-1))
            xoff[k] = off
            off += r.numel() * data.d
        Xrs = torch.cat(blocks) if blocks else torch.zeros(1, device=dev)
        norm2 = {k: (data.X[rowsets[k]].double() ** 2).sum(1) for k in keys}
        # ---- problems --------------------------------------------------------------------
        probs, prob_of, ys, Cs, Gs, qds = [], [], [], [], [], []
        voff = roff = koff = 0
        gammas: Dict[int, float] = {}
        for ti, t in enumerate(tasks):
            rp = t.params
            gamma = self._gamma(data, t, rp["gamma"], gammas)
            for pi, pr in enumerate(pairs):
                key = (t.split, pr)
                rows = rowsets[key]
                nr = rows.numel()
                if nr == 0:
                    continue
                if svr:
                    yv = data.y_reg[rows].double()
                    L = 2 * nr
                    y_t = torch.cat([torch.ones(nr), -torch.ones(nr)]).to(dev)
                    G0 = torch.cat([rp["epsilon"] - yv, rp["epsilon"] + yv])
                    C_t = torch.full((L,), rp["C"], dtype=torch.float64, device=dev)
                else:
                    cls = data.y_cls[rows]
                    L = nr
                    y_t = torch.where(cls == pr[0], 1.0, -1.0).to(dev)
                    G0 = torch.full((L,), -1.0, dtype=torch.float64, device=dev)
                    w = self._class_weights(data, t, rp["class_weight"])
                    C_t = rp["C"] * torch.where(cls == pr[0], w[pr[0]], w[pr[1]]).double()
                qd = self._diag(norm2[key], rp["kernel"], gamma, rp["coef0"], rp["degree"])
                mi = rp["max_iter"] if rp["max_iter"] > 0 else max(10_000_000, 100 * L)
                probs.append((xoff[key], roff, nr, L, voff, koff, rp["kernel"], rp["degree"], gamma, rp["coef0"],
                              rp["tol"], mi, 0, 0, int(svr), 0, 0))
                prob_of.append((ti, pi, key))
                ys.append(y_t.float()); Cs.append(C_t); Gs.append(G0); qds.append(qd.float())
                voff += L; roff += nr; koff += 2 * nr
        P = np.array(probs, dtype=PROB_DTYPE)
        y_all = torch.cat(ys).float().contiguous()
        C_all = torch.cat(Cs).double().contiguous()
        G_all = torch.cat(Gs).double().contiguous()
        qd_all = torch.cat(qds).float().contiguous()
        a_all = torch.zeros_like(G_all)
        self._solve(data, P, Xrs, y_all, C_all, qd_all, a_all, G_all, koff)
        # ---- rho, decision values, predictions --------------------------------------------
        dec: Dict[Tuple[int, int], torch.Tensor] = {}
        models: Dict[int, list] = {}
        for k, (ti, pi, key) in enumerate(prob_of):
            t = tasks[ti]
            rec = P[k]
            v0, L, nr = int(rec["voff"]), int(rec["L"]), int(rec["nrows"])
            a = a_all[v0:v0 + L]
            g = G_all[v0:v0 + L]
            y = y_all[v0:v0 + L].double()
            Cv = C_all[v0:v0 + L]
            rho = _rho(a, g, y, Cv)
            coef = (a[:nr] - a[nr:]) if svr else a * y
            sv = coef != 0
            rows = rowsets[key]
            Xsv = data.X[rows[sv]]
            te = data.test_rows[t.split].long()
            K = _kernel_matrix(data.X[te], Xsv, int(rec["kernel"]), float(rec["gamma"]), float(rec["coef0"]),
                               int(rec["degree"]))
            dec[(ti, pi)] = K @ coef[sv].to(K.dtype) - rho
            if keep_models:
                models.setdefault(ti, []).append({"sv": Xsv.cpu().numpy(), "coef": coef[sv].cpu().numpy(),
                                                  "rho": float(rho), "pair": pairs[pi]})
            if int(rec["status"]) == 2:
                w = f"Solver terminated early (max_iter={int(rec['max_iter'])})"
                if w not in t.params["warnings"]:
                    t.params["warnings"].append(w)
        data.sync()
        dt = time.perf_counter() - t0
        outs = []
        for ti, t in enumerate(tasks):
            te = data.test_rows[t.split]
            if svr:
                pred = dec[(ti, 0)].float() if (ti, 0) in dec else torch.zeros(te.numel(), device=dev)
            else:
                votes = torch.zeros((te.numel(), C_cls), dtype=torch.int32, device=dev)
                for pi, (a_, b_) in enumerate(pairs):
                    dv = dec.get((ti, pi))
                    if dv is None:
                        continue
                    votes[:, a_] += (dv > 0).int()
                    votes[:, b_] += (dv <= 0).int()
                pred = votes.argmax(1).to(torch.int32)      # first max = lowest class (libsvm vote)
                if t.params.get("break_ties") and C_cls > 2:
                    pred = _ovr_argmax(dec, ti, pairs, te.numel(), C_cls, dev)
            o = FitOutput(task_id=t.task_id, pred=pred, fit_seconds=dt / len(tasks),
                          info={"warnings": t.params["warnings"]})
            if not svr and C_cls == 2 and (ti, 0) in dec:
                o.decision = -dec[(ti, 0)]   # sklearn's binary decision_function: positive -> classes_[1]
            if keep_models:
                rp = t.params
                o.model = {"kind": "svm", "svr": svr, "machines": models.get(ti, []), "kernel": rp["kernel"],
                           "gamma": float(self._gamma(data, t, rp["gamma"], {})), "coef0": rp["coef0"],
                           "degree": rp["degree"], "n_classes": C_cls,
                           "classes": None if svr else np.asarray(data.classes).tolist(), "model_type": t.model_type}
            outs.append(o)
        return outs

    def _solve(self, data, P, Xrs, y, C, qd, alpha, G, kbuf_len):
        if data.is_gpu:
            lib = native.hip_lib()
            if lib.dml_svm_sizeof_prob() != PROB_DTYPE.itemsize:
                raise RuntimeError("SvmProb layout mismatch")
            if os.environ.get("DML_SVM_SPLIT", "1") != "0" and self._solve_split(data, lib, P, Xrs, y, C, qd, alpha, G):
                return
            kbuf = torch.empty(max(1, kbuf_len), dtype=torch.float32, device=data.device)
            Pd = torch.from_numpy(P.view(np.uint8).copy()).to(data.device)
            while True:
                rc = lib.dml_svm_smo(native.ptr(Xrs), data.d, native.ptr(Pd), len(P), native.ptr(y), native.ptr(C),
                                     native.ptr(qd), native.ptr(alpha), native.ptr(G), native.ptr(kbuf), CHUNK_ITERS,
                                     native.stream_handle(data.device))
                if rc:
                    raise RuntimeError("dml_svm_smo launch failed")
                P[:] = Pd.cpu().numpy().view(PROB_DTYPE)
                if (P["status"] != 0).all():
                    break
            self.last_solve_stats = {"solver": "one workgroup per problem", "problems": len(P),
                                     "iterations_max": int(P["iters"].max())}
        else:
            lib = native.cpu_lib()
            if lib.dml_cpu_svm_sizeof_prob() != PROB_DTYPE.itemsize:
                raise RuntimeError("SvmProb layout mismatch")
            lib.dml_cpu_svm_smo(native.ptr(Xrs), data.d, native.ptr(P), len(P), native.ptr(y), native.ptr(C),
                                native.ptr(qd), native.ptr(alpha), native.ptr(G))

    def _solve_split(self, data, lib, P, Xrs, y, C, qd, alpha, G) -> bool:
        """B workgroups per problem + per-problem LRU kernel-column caches
        (csrc/kernels/svm.hip ``k_smo_split``).  Every launch (a chunk of SMO iterations)
        re-splits the still-running problems over the resident workgroups, so the last
        hard problems (large C) end up with the most workgroups.  False: the split solver
        cannot run here (the caller uses the one-workgroup kernel)."""
        dev = data.device
        nprob = len(P)
        max_b, max_slots, wide_res = ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_int32(0)
        resident = int(lib.dml_svm_split_limits(ctypes.byref(max_b), ctypes.byref(max_slots), ctypes.byref(wide_res)))
        wide_ok = os.environ.get("DML_SVM_WIDE", "1") != "0"
        nr = P["nrows"].astype(np.int64)
        if resident <= 0 or nprob == 0:
            return False
        MB = int(max_b.value)
        free = torch.cuda.mem_get_info(dev)[0]
        cache_bytes = min(CACHE_FRACTION * free, float(os.environ.get("DML_SVM_CACHE_GB", CACHE_MAX_GB)) * 1e9)
        S = int(min(max_slots.value, int(nr.max()), cache_bytes // max(1, 4 * int(nr.sum()))))
        if os.environ.get("DML_SVM_CACHE_SLOTS"):   # tests: force evictions
            S = min(S, int(os.environ["DML_SVM_CACHE_SLOTS"]))
        if S < 2:
            return False
        P["coff"] = np.concatenate([[0], np.cumsum(nr * S)[:-1]])
        rep = nr + 2 * S                               # one workgroup's map: slot_of [nr], row_of [S], stamp [S]
        P["moff"] = np.concatenate([[0], np.cumsum(MB * rep)[:-1]])
        meta_np = np.full(int((MB * rep).sum()), -1, dtype=np.int32)
        for p in range(nprob):   # stamps start at 0: unused slots are the first victims
            for w in range(MB):
                st = int(P["moff"][p]) + w * int(rep[p]) + int(nr[p]) + S
                meta_np[st:st + S] = 0
        meta = torch.from_numpy(meta_np).to(dev)
        kc = torch.empty(int((nr * S).sum()), dtype=torch.float32, device=dev)
        prof = torch.zeros(8, dtype=torch.int64, device=dev) if os.environ.get("DML_SVM_PROFILE") else None
        launches, B_prev, B_hist, wide_n = 0, 0, [], 0
        while True:
            run = np.nonzero(P["status"] == 0)[0]
            if run.size == 0:
                break
            B = int(min(MB, max(1, resident // run.size), max(1, int(nr[run].max()) // MIN_ROWS_PER_WG)))
            if run.size * B > resident:
                B = 1   # no cross-workgroup waits at B = 1: any grid size is safe
            if launches and B != B_prev:
                # every replica of a problem's cache map is identical and every cached column
                # is complete (the old slices covered all rows): copy replica 0 to the new ones
                for p in run:
                    o, r_ = int(P["moff"][p]), int(rep[p])
                    view = meta[o:o + MB * r_].view(MB, r_)
                    view[1:B] = view[0]
            Pr = np.ascontiguousarray(P[run])
            Pd = torch.from_numpy(Pr.view(np.uint8).copy()).to(dev)
            recs = torch.zeros(run.size * 2 * B * 12, dtype=torch.int64, device=dev)   # svm.hip kRecW
            out_state = torch.zeros(2 * run.size, dtype=torch.int64, device=dev)
            # the wide sweep (8 variables per thread per step: one round trip per sweep for a
            # slice of <= 2048 rows) once the remaining problems fit its lower occupancy
            wide = int(wide_ok and (B == 1 or run.size * B <= int(wide_res.value))
                       and int(nr[run].max()) <= 8 * 256 * B)
            rc = lib.dml_svm_smo_split(native.ptr(Xrs), data.d, native.ptr(Pd), run.size, B, S, native.ptr(y),
                                       native.ptr(C), native.ptr(qd), native.ptr(alpha), native.ptr(G), native.ptr(kc),
                                       native.ptr(meta), native.ptr(recs), native.ptr(out_state), SPLIT_CHUNK_ITERS,
                                       native.ptr(prof), wide, native.stream_handle(dev))
            if rc == 4 and launches == 0:
                return False
            if rc:
                raise RuntimeError(f"dml_svm_smo_split failed ({rc})")
            launches += 1
            wide_n += wide
            B_prev = B
            B_hist.append(B)
            st = out_state.view(run.size, 2).cpu().numpy()
            P["iters"][run] = st[:, 0]
            P["status"][run] = st[:, 1]
            if (P["status"] == 3).any():
                raise RuntimeError("SMO workgroups of a problem lost contact (not co-resident?)")
        self.last_solve_stats = {"solver": "split", "problems": nprob, "workgroups_per_problem": max(B_hist),
                                 "wide_launches": wide_n,
                                 "workgroups_per_launch": B_hist, "cache_slots": S, "launches": launches,
                                 "iterations_max": int(P["iters"].max()), "iterations_sum": int(P["iters"].sum())}
        if prof is not None:   # first running problem, workgroup 0: 100 MHz ticks -> microseconds per phase
            pr = prof.cpu().numpy()
            names = ("i_reduce", "xchg_i", "col_i", "j_sweep", "xchg_j", "col_j_update", "g_sweep")
            self.last_solve_stats["phase_us"] = {k: round(float(pr[q]) / 100.0, 1) for q, k in enumerate(names)}
            self.last_solve_stats["cache_misses"] = int(pr[7])
        return True

    @staticmethod
    def _gamma(data, t: FitTask, gamma, cache: Dict[int, float]) -> float:
        if not isinstance(gamma, str):
            return float(gamma)
        if gamma == "auto":
            return 1.0 / data.d
        if t.split not in cache:
            Xt = data.X[data.train_rows[t.split].long()].double()
            var = float(Xt.var(unbiased=False)) if Xt.numel() else 0.0
            cache[t.split] = 1.0 / (data.d * var) if var != 0 else 1.0
        return cache[t.split]

    @staticmethod
    def _class_weights(data, t: FitTask, cw) -> torch.Tensor:
        C = data.n_classes
        w = torch.ones(C, dtype=torch.float64, device=data.device)
        if cw is None:
            return w
        if cw == "balanced":
            yt = data.y_cls[data.train_rows[t.split].long()].long()
            cnt = torch.bincount(yt, minlength=C).double()
            return torch.where(cnt > 0, yt.numel() / (C * cnt.clamp_min(1)), torch.ones_like(cnt))
        lookup = {str(c): i for i, c in enumerate(np.asarray(data.classes).tolist())}
        for k, v in cw.items():
            if str(k) in lookup:
                w[lookup[str(k)]] = float(v)
        return w

    @staticmethod
    def _diag(norm2: torch.Tensor, kernel: int, gamma: float, coef0: float, degree: int) -> torch.Tensor:
        if kernel == KRBF:
            return torch.ones_like(norm2)
        if kernel == KLIN:
            return norm2
        if kernel == KPOLY:
            return (gamma * norm2 + coef0) ** degree
        return torch.tanh(gamma * norm2 + coef0)


def _rho(a, g, y, C) -> float:
    """libsvm Solver::calculate_rho."""
    yG = y * g
    upper = a >= C
    lower = a <= 0
    free = ~upper & ~lower
    if bool(free.any()):
        return float(yG[free].mean())
    ub_mask = (upper & (y < 0)) | (lower & (y > 0))
    lb_mask = (upper & (y > 0)) | (lower & (y < 0))
    ub = float(yG[ub_mask].min()) if bool(ub_mask.any()) else math.inf
    lb = float(yG[lb_mask].max()) if bool(lb_mask.any()) else -math.inf
    return (ub + lb) / 2


def _kernel_matrix(A: torch.Tensor, B: torch.Tensor, kernel: int, gamma: float, coef0: float, degree: int):
    dt = torch.float64 if A.shape[0] * max(1, B.shape[0]) <= 50_000_000 else torch.float32
    A, B = A.to(dt), B.to(dt)
    if kernel == KRBF:
        d2 = (A * A).sum(1, keepdim=True) + (B * B).sum(1)[None, :] - 2.0 * (A @ B.t())
        return torch.exp(-gamma * d2.clamp_min(0))
    dot = A @ B.t()
    if kernel == KLIN:
        return dot
    if kernel == KPOLY:
        return (gamma * dot + coef0) ** degree
    return torch.tanh(gamma * dot + coef0)


def svm_predict_numpy(model: Dict[str, Any], X: np.ndarray) -> np.ndarray:
    Xt = torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32))
    decs = []
    for m in model["machines"]:
        sv = torch.from_numpy(np.asarray(m["sv"], dtype=np.float32).reshape(-1, Xt.shape[1]))
        K = _kernel_matrix(Xt, sv, int(model["kernel"]), float(model["gamma"]), float(model["coef0"]),
                           int(model["degree"]))
        decs.append((K @ torch.from_numpy(np.asarray(m["coef"], dtype=np.float64)).to(K.dtype) - m["rho"]).numpy())
    if model["svr"]:
        return decs[0] if decs else np.zeros(len(X))
    C = int(model["n_classes"])
    votes = np.zeros((len(X), C), dtype=np.int64)
    for m, dv in zip(model["machines"], decs):
        a, b = m["pair"]
        votes[:, a] += dv > 0
        votes[:, b] += dv <= 0
    return np.asarray(model["classes"])[votes.argmax(1)]


register(SVMFamily())
