"""Row-sharded (data-parallel) forest builder: per-level histogram all-reduce.

SURVEY §2.7 / §5.7(b) / §5.8 "DP mode" for random forests: every rank holds one
contiguous row block of the table (``parallel/data_parallel.py`` RowShard) and the trees
of a batch grow level-synchronously on ALL ranks at once:

1. each rank histograms the open nodes of the level over its own rows
   (``csrc/kernels/forest_dp.hip``: LDS-privatised tiles for large nodes, global atomics
   for small ones; the C++ twin ``csrc/runtime/forest_dp_cpu.cpp`` on CPU);
2. ONE reduce-scatter per level-round sums the ``[nodes, positions, channels, 256]``
   histogram tensor over the ranks, split by node (RCCL over xGMI; gloo on CPU): each
   rank owns 1/N of the nodes' global histograms;
3. each rank evaluates its own nodes with the shared code (``forest_dp.h``) and one
   all-gather of the 64-B decision records gives every rank every decision, so every rank
   holds the same node pool; each partitions only its own (tree, row) pairs, which are
   re-sorted by node for the next level.

The reference has no counterpart: its workers each re-read the whole CSV and fit one
candidate alone (aws-prod/worker/worker.py:406-425, :315).  Decisions follow the one-GPU
builders exactly (bootstrap weight of the GLOBAL row id, keyed per-node feature order,
max_features non-constant search, first-strictly-better ties), so a row-sharded
classification forest is the forest ``forest_ops.build_gpu`` / ``build_cpu`` grows.

Cost per level-round over xGMI: open nodes x KR positions x channels x 1 KiB (int32
counts); e.g. 2,048 nodes x 10 x 3 channels = 60 MB.  Deep levels of full-depth trees
have many small nodes, so the mode is meant for what SURVEY §5.7 names: tables larger
than one GPU's HBM (and bounded-depth or min_samples_leaf-limited trees); the default
task-parallel path stays the fast one when every rank can hold the table.
"""
from __future__ import annotations

import ctypes
import os
import time
from typing import Callable, Optional

import numpy as np
import torch

from ..utils import native, trace
from .forest_ops import reg_exponent_counts, reg_exponents_of_counts, _n_targets, ForestBuild

SLOT_BYTES = 64
# int32 column of each DpSlot field (forest_dp.h): key 0-1, best_gain 2-3, count 4-5
F_NODE, F_TREE, F_DEPTH, F_POS, F_NONCONST, F_FEAT, F_BIN, F_DONE, F_SPLIT, F_CHILD = range(6, 16)

SMALL_SEG = 1024         # pairs: below this a node's histogram goes straight to global atomics
TILE_ROWS = 4096         # pairs per LDS tile of a large node
LDS_BYTES = 65536        # LDS per workgroup for the tile histograms
HIST_BUDGET = 1 << 30    # bytes of histogram per all-reduce chunk
# classification nodes of <= this many global rows exchange sparse histograms: a row adds
# at most 2 x KR non-zero (index, count) int32 pairs (8 B each) against the node's dense
# KR x channels x 1 KiB reduce-scatter share.  Swept on a 2-rank gloo build (60k x 20,
# 8 full-depth trees): exchanged bytes 0.38 GB dense -> 0.20 / 0.135 / 0.121 GB at
# 16 / 48 / 96 rows (profiles/r2_forest_dp_sparse_sweep.log)
SPARSE_ROWS = 96


class DpArgs(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in (
        "Xb ld n d r0 ycls yreg C CH VC is_reg roles specs T cw tree_W root wts "
        "act_row act_tree act_node A new_node slots best_left S_open seg_start seg_cnt "
        "srch S KR feats hist tile_s tile_off n_tiles tile_rows small_s n_small lds_feats "
        "nodes vals P child_base next next_open slot_of lvl_lo lvl_n hi binvals exact P_total ystride yq_e1 yq_e2").split()]


Reducer = Callable[[torch.Tensor, str], torch.Tensor]   # (tensor, "sum" | "min" | "max") -> in place


def _no_reduce(t: torch.Tensor, op: str = "sum") -> torch.Tensor:
    return t


class _Lib:
    def __init__(self, dev: torch.device):
        self.gpu = dev.type == "cuda"
        self.dev = dev
        if self.gpu:
            self.lib = native.hip_lib()
            if self.lib.dml_dp_sizeof_args() != ctypes.sizeof(DpArgs) or self.lib.dml_dp_sizeof_slot() != SLOT_BYTES:
                raise RuntimeError("DpArgs / DpSlot layout mismatch between HIP library and Python")
        else:
            self.lib = native.cpu_lib()
            if self.lib.dml_cpu_dp_sizeof_args() != ctypes.sizeof(DpArgs):
                raise RuntimeError("DpArgs layout mismatch between C++ library and Python")

    def step(self, a: DpArgs, step: int) -> None:
        if self.gpu:
            rc = self.lib.dml_dp_step(ctypes.byref(a), step, native.stream_handle(self.dev))
        else:
            rc = self.lib.dml_cpu_dp_step(ctypes.byref(a), step)
        if rc:
            raise RuntimeError(f"forest DP step {step} failed ({rc})")


def _p(t) -> int:
    return 0 if t is None else int(t.data_ptr())


def _build_chunk(Xb: torch.Tensor, ycls: Optional[torch.Tensor], yreg: Optional[torch.Tensor], roles: torch.Tensor,
                 specs: np.ndarray, n_classes: int, is_reg: bool, r0: int, reduce: Reducer = _no_reduce,
                 cw: Optional[np.ndarray] = None, hist_budget: int = HIST_BUDGET, comm=None,
                 ystride: int = 0) -> ForestBuild:
    """One level-synchronous build of every tree of ``specs`` (``build_dp`` documents the
    arguments and the collectives)."""
    dev = Xb.device
    L = _Lib(dev)
    t0 = time.perf_counter()
    n, d = Xb.shape
    T = len(specs)
    C = 1 if is_reg else int(n_classes)
    CH, VC = (4, 3) if is_reg else (C + 1, C)
    a = DpArgs()
    a.Xb, a.ld, a.n, a.d, a.r0 = _p(Xb), Xb.stride(0), n, d, int(r0)
    a.ycls, a.yreg, a.ystride = _p(ycls), _p(yreg), int(ystride)
    a.C, a.CH, a.VC, a.is_reg = C, CH, VC, int(is_reg)
    roles = roles.contiguous()
    a.roles = _p(roles)
    specs_dev = torch.from_numpy(np.ascontiguousarray(specs).view(np.uint8).copy()).to(dev)
    a.specs, a.T = _p(specs_dev), T
    cw_t = None
    if cw is not None and not is_reg:
        cw_t = torch.from_numpy(np.ascontiguousarray(cw, dtype=np.float64).reshape(T, C)).to(dev)
    a.cw = _p(cw_t)
    mf = torch.from_numpy(np.ascontiguousarray(specs["max_features"], dtype=np.int32)).to(dev)
    stats = {"levels": 0, "rounds": 0, "allreduce_bytes": 0, "hist_s": 0.0, "reduce_s": 0.0}

    if is_reg:
        # the fixed-point exponents of the ONE-GPU build of the whole table: the targets'
        # exponent histograms summed over every rank (exact counts, forest_common.h
        # reg_exponents_counts)
        targets = _n_targets(specs, ystride)
        cnt = reg_exponent_counts(yreg, n, ystride, targets).to(torch.float64)
        a.yq_e1, a.yq_e2 = reg_exponents_of_counts(reduce(cnt.reshape(-1).clone(), "sum").round().to(torch.int64))
    # ---- roots: local bootstrap statistics, summed over the ranks ----------------------
    wts = torch.empty((T, n), dtype=torch.uint8, device=dev)
    a.wts = _p(wts)
    L.step(a, 0)
    # regression roots are exact integer sums {w, w yq, w y2q, rows}
    root = torch.zeros((T, CH), dtype=torch.int64 if is_reg else torch.float64, device=dev)
    a.root = _p(root)
    L.step(a, 1)
    reduce(root, "sum")
    cap = max(1024, 8 * T)
    nodes = torch.empty((cap, 2), dtype=torch.int32, device=dev)
    vals = torch.zeros((cap, VC), dtype=torch.float64, device=dev)
    tree_W = torch.empty(T, dtype=torch.float64, device=dev)
    nxt = torch.empty((T, SLOT_BYTES), dtype=torch.uint8, device=dev)
    nxt_open = torch.empty(T, dtype=torch.int32, device=dev)
    a.nodes, a.vals, a.tree_W, a.next, a.next_open = _p(nodes), _p(vals), _p(tree_W), _p(nxt), _p(nxt_open)
    L.step(a, 2)
    open_t = nxt_open.bool()
    slots = nxt[open_t].contiguous()
    pair = torch.nonzero(((wts > 0) & open_t[:, None]).reshape(-1)).flatten()
    del wts
    act_tree = (pair // n).to(torch.int32)
    act_row = (pair - act_tree.to(torch.int64) * n).to(torch.int32)
    act_node = act_tree.clone()           # tree t's root is node t; pairs already sorted by node
    del pair
    P, lvl_lo, lvl_n = T, 0, T
    # regression: three integer planes (w | rows << 32, w yq, w y2q), u64 as int64
    hist_dtype = torch.int64 if is_reg else torch.int32
    HP = 3 if is_reg else CH
    pos_bytes = HP * 256 * (8 if is_reg else 4)      # histogram bytes of one visiting position
    world = int(getattr(comm, "world", 1)) if comm is not None else 1
    scatter = world > 1
    lds_feats = LDS_BYTES // pos_bytes
    timing = os.environ.get("DML_DP_TIMING") == "1"

    while slots.shape[0]:
        S_open = int(slots.shape[0])
        sv = slots.view(torch.int32)
        slot_nodes = sv[:, F_NODE].contiguous()
        seg_start = torch.searchsorted(act_node, slot_nodes).to(torch.int64)
        seg_cnt = torch.searchsorted(act_node, slot_nodes, right=True).to(torch.int64) - seg_start
        best_left = torch.zeros((S_open, CH), dtype=torch.float64, device=dev)
        a.act_row, a.act_tree, a.act_node, a.A = _p(act_row), _p(act_tree), _p(act_node), int(act_row.numel())
        a.slots, a.best_left, a.S_open = _p(slots), _p(best_left), S_open
        a.seg_start, a.seg_cnt = _p(seg_start), _p(seg_cnt)
        # ---- the feature search, round by round -----------------------------------------
        while True:
            srch = torch.nonzero(sv[:, F_DONE] == 0).flatten().to(torch.int32)
            S = int(srch.numel())
            if S == 0:
                break
            sl = srch.long()
            need = int((mf[sv[sl, F_TREE].long()] - sv[sl, F_NONCONST]).max())
            left_pos = int((d - sv[sl, F_POS]).max())
            KR = max(1, min(left_pos, need + max(1, need // 4)))
            chunk = max(1, hist_budget // (KR * pos_bytes))
            # small nodes of a classification forest exchange sparse local histograms
            # (non-zero (index, count) pairs) instead of dense 256-bin tensors
            groups = [(srch, False)]
            if scatter and not is_reg:
                small_n = slots.view(torch.float64)[sl, 2] <= SPARSE_ROWS
                groups = [(srch[~small_n].contiguous(), False), (srch[small_n].contiguous(), True)]
            for grp, sparse in groups:
                Sg = int(grp.numel())
                for c0 in range(0, Sg, chunk):
                    sub = grp[c0:c0 + chunk].contiguous()
                    Sc = int(sub.numel())
                    feats = torch.empty((Sc, KR), dtype=torch.int32, device=dev)
                    q = -(-Sc // world)                          # nodes owned per rank (reduce-scatter)
                    rs = scatter and not sparse
                    hist = torch.zeros((q * world if rs else Sc, KR, HP, 256), dtype=hist_dtype, device=dev)
                    a.srch, a.S, a.KR, a.feats, a.hist = _p(sub), Sc, KR, _p(feats), _p(hist)
                    L.step(a, 3)
                    th = time.perf_counter()
                    cnt = seg_cnt[sub.long()]
                    if L.gpu and lds_feats > 0:
                        big = cnt >= SMALL_SEG
                        bi = torch.nonzero(big).flatten()
                        nt = (cnt[bi] + TILE_ROWS - 1) // TILE_ROWS
                        n_tiles = int(nt.sum()) if bi.numel() else 0
                        tile_s = torch.repeat_interleave(bi.to(torch.int32), nt, output_size=n_tiles)
                        first = torch.cumsum(nt, 0) - nt
                        tile_off = (torch.arange(n_tiles, device=dev) -
                                    torch.repeat_interleave(first, nt, output_size=n_tiles)) * TILE_ROWS
                        small = torch.nonzero((~big) & (cnt > 0)).flatten().to(torch.int32)
                    else:
                        tile_s = tile_off = None
                        n_tiles = 0
                        small = torch.nonzero(cnt > 0).flatten().to(torch.int32)
                    a.tile_s, a.tile_off, a.n_tiles, a.tile_rows = _p(tile_s), _p(tile_off), n_tiles, TILE_ROWS
                    a.small_s, a.n_small, a.lds_feats = _p(small), int(small.numel()), max(1, min(lds_feats, KR))
                    with trace.range("forest_dp_hist"):
                        L.step(a, 4)
                        if L.gpu and timing:   # per-phase timing only: the collective orders itself
                            torch.cuda.current_stream(dev).synchronize()
                    tr = time.perf_counter()
                    stats["hist_s"] += tr - th
                    if sparse:
                        # every rank sums the same gathered (index, count) pairs: integer
                        # sums, identical on every rank, so every rank evaluates these nodes
                        with trace.range("forest_dp_sparse_gather"):
                            flat = hist.view(-1)
                            nz = torch.nonzero(flat).flatten()
                            pairs = torch.stack([nz.to(torch.int32), flat[nz].to(torch.int32)], 1)   # < 2^28 bins
                            cnts = comm.all_gather_equal(torch.tensor([pairs.shape[0]], dtype=torch.int64, device=dev))
                            m = int(cnts.max())          # the same on every rank
                            if m > 0:
                                pad = torch.zeros((m, 2), dtype=torch.int32, device=dev)
                                pad[:pairs.shape[0]] = pairs
                                allp = comm.all_gather_equal(pad)
                                keep = torch.cat([torch.arange(m, device=dev) < int(c) for c in cnts.tolist()])
                                allp = allp[keep]
                                flat.zero_()
                                flat.index_add_(0, allp[:, 0].long(), allp[:, 1].to(hist_dtype))
                        stats["reduce_s"] += time.perf_counter() - tr
                        stats["allreduce_bytes"] += int(cnts.sum()) * 8
                        L.step(a, 5)
                    elif scatter:
                        # owner-computes: the global sums of this rank's 1/N of the nodes
                        with trace.range("forest_dp_reduce_scatter"):
                            own = comm.reduce_scatter_rows(hist)
                        stats["reduce_s"] += time.perf_counter() - tr
                        stats["allreduce_bytes"] += hist.numel() * hist.element_size() // 2   # ring: half an all-reduce
                        lo = min(Sc, comm.rank * q)
                        hi = min(Sc, lo + q)
                        own_srch = sub[lo:hi].contiguous()
                        a.srch, a.S, a.hist, a.feats = _p(own_srch), hi - lo, _p(own), _p(feats[lo:hi])
                        L.step(a, 5)
                        idx = own_srch.long()
                        rec = torch.zeros((q, SLOT_BYTES + 8 * CH), dtype=torch.uint8, device=dev)
                        rec[:hi - lo, :SLOT_BYTES] = slots[idx]
                        rec[:hi - lo, SLOT_BYTES:] = best_left[idx].view(torch.uint8)
                        with trace.range("forest_dp_gather_decisions"):
                            rec = comm.all_gather_equal(rec)[:Sc]
                        sl_all = sub.long()
                        slots[sl_all] = rec[:, :SLOT_BYTES]
                        best_left[sl_all] = rec[:, SLOT_BYTES:].contiguous().view(torch.float64)
                        a.srch, a.S, a.hist, a.feats = _p(sub), Sc, _p(hist), _p(feats)
                    else:
                        with trace.range("forest_dp_allreduce"):
                            reduce(hist, "sum")
                        stats["reduce_s"] += time.perf_counter() - tr
                        stats["allreduce_bytes"] += hist.numel() * hist.element_size()
                        L.step(a, 5)
                    stats["rounds"] += 1
                    del feats, hist, tile_s, tile_off, small
        # ---- accept, children, partition ------------------------------------------------
        L.step(a, 6)
        split = sv[:, F_SPLIT]
        n_split = int(split.sum())
        stats["levels"] += 1
        if n_split == 0:
            break
        child_base = ((torch.cumsum(split, 0) - split) * 2).to(torch.int32)
        if P + 2 * n_split > cap:
            cap = max(2 * cap, P + 2 * n_split)
            nodes2 = torch.empty((cap, 2), dtype=torch.int32, device=dev)
            vals2 = torch.zeros((cap, VC), dtype=torch.float64, device=dev)
            nodes2[:P] = nodes[:P]
            vals2[:P] = vals[:P]
            nodes, vals = nodes2, vals2
            a.nodes, a.vals = _p(nodes), _p(vals)
        nxt = torch.empty((2 * n_split, SLOT_BYTES), dtype=torch.uint8, device=dev)
        nxt_open = torch.empty(2 * n_split, dtype=torch.int32, device=dev)
        a.P, a.child_base, a.next, a.next_open = P, _p(child_base), _p(nxt), _p(nxt_open)
        L.step(a, 7)
        slot_of = torch.full((lvl_n,), -1, dtype=torch.int32, device=dev)
        slot_of[(slot_nodes - lvl_lo).long()] = torch.arange(S_open, dtype=torch.int32, device=dev)
        new_node = torch.empty(max(1, int(act_row.numel())), dtype=torch.int32, device=dev)
        a.slot_of, a.lvl_lo, a.lvl_n, a.new_node = _p(slot_of), lvl_lo, lvl_n, _p(new_node)
        L.step(a, 8)
        new_node = new_node[:act_row.numel()]
        keep = new_node >= 0
        act_node, perm = torch.sort(new_node[keep], stable=True)
        act_row = act_row[keep][perm].contiguous()
        act_tree = act_tree[keep][perm].contiguous()
        act_node = act_node.contiguous()
        slots = nxt[nxt_open.bool()].contiguous()
        lvl_lo, lvl_n = P, 2 * n_split
        P += 2 * n_split
    stats.update(nodes=P, build_s=time.perf_counter() - t0)
    fb = ForestBuild(nodes[:P], vals[:P], T, VC, is_reg, int(n_classes), stats)
    fb.dp_specs_dev = specs_dev
    return fb


def build_dp(Xb: torch.Tensor, ycls: Optional[torch.Tensor], yreg: Optional[torch.Tensor], roles: torch.Tensor,
             specs: np.ndarray, n_classes: int, is_reg: bool, r0: int, reduce: Reducer = _no_reduce,
             cw: Optional[np.ndarray] = None, hist_budget: int = HIST_BUDGET, comm=None,
             ystride: int = 0, tree_chunk: Optional[int] = None) -> ForestBuild:
    """Grow the ``specs`` trees over the row shard ``Xb`` (global rows ``r0 ..``);
    ``reduce`` sums / mins tensors over the ranks.  Every rank returns the same pool.

    ``comm`` (world > 1; ``RowShard`` provides it): ``reduce_scatter_rows`` /
    ``all_gather_equal`` / ``rank`` / ``world``.  Each level-round's histograms are then
    REDUCE-SCATTERED by node: rank k receives the global sums of 1/N of the searching
    nodes only, evaluates just those, and one all-gather of the (64 B slot + best-left
    sums) records makes every rank's decisions identical again.  Over a ring that moves
    half the bytes of an all-reduce, and the split evaluation is divided by N.

    ``tree_chunk``: grow at most this many trees at a time (the (tree, row) pair arrays
    cost ~26 B per tree and local row: a 1000-tree fit on a 25M-row shard would need
    650 GB at once); the chunks' pools are concatenated into the one-build layout."""
    T = len(specs)
    tc = T if not tree_chunk else max(1, min(T, int(tree_chunk)))
    if tc >= T:
        return _build_chunk(Xb, ycls, yreg, roles, specs, n_classes, is_reg, r0, reduce, cw, hist_budget, comm,
                            ystride)
    parts = []
    for t0 in range(0, T, tc):
        t1 = min(T, t0 + tc)
        parts.append(_build_chunk(Xb, ycls, yreg, roles, specs[t0:t1], n_classes, is_reg, r0, reduce,
                                  None if cw is None else np.ascontiguousarray(cw[t0:t1]), hist_budget, comm,
                                  ystride))
    return _concat_pools(parts, T)


def _concat_pools(parts, T: int) -> ForestBuild:
    """Pools of consecutive tree chunks -> one pool in the builders' layout (tree t's root
    at node t, every other node after the roots, child pairs adjacent)."""
    dev = parts[0].nodes.device
    P_total = T + sum(int(p.nodes.shape[0]) - p.n_trees for p in parts)
    nodes = torch.empty((P_total, 2), dtype=torch.int32, device=dev)
    vals = torch.empty((P_total, parts[0].VC), dtype=torch.float64, device=dev)
    root_base, rest = 0, T
    stats = {}
    for p in parts:
        Pc, Tc = int(p.nodes.shape[0]), p.n_trees
        m = torch.empty(Pc, dtype=torch.int64, device=dev)
        m[:Tc] = torch.arange(root_base, root_base + Tc, device=dev)
        m[Tc:] = torch.arange(rest, rest + Pc - Tc, device=dev)
        nd = p.nodes.clone()
        internal = nd[:, 1] >= 0
        nd[internal, 1] = m[nd[internal, 1].long()].to(torch.int32)
        nodes[m] = nd
        vals[m] = p.vals
        root_base += Tc
        rest += Pc - Tc
        for k, v in p.stats.items():
            if isinstance(v, (int, float)):
                stats[k] = stats.get(k, 0) + v
    stats["nodes"] = P_total
    stats["tree_chunks"] = len(parts)
    fb = ForestBuild(nodes, vals, T, parts[0].VC, parts[0].is_reg, parts[0].n_classes, stats)
    fb.dp_specs_dev = None
    return fb


def refine_dp(fb: ForestBuild, Xb: torch.Tensor, roles: torch.Tensor, specs: np.ndarray, r0: int,
              binvals: torch.Tensor, exact: torch.Tensor, reduce: Reducer = _no_reduce) -> None:
    """sklearn midpoint thresholds on exactly-binned features (in place): the smallest
    right-going bin per node is a MIN over every rank's training rows."""
    dev = Xb.device
    L = _Lib(dev)
    P = int(fb.nodes.shape[0])
    a = DpArgs()
    specs_dev = torch.from_numpy(np.ascontiguousarray(specs).view(np.uint8).copy()).to(dev)
    roles = roles.contiguous()
    hi = torch.full((P,), 0x7FFFFFFF, dtype=torch.int32, device=dev)
    a.Xb, a.ld, a.n, a.d, a.r0 = _p(Xb), Xb.stride(0), Xb.shape[0], Xb.shape[1], int(r0)
    a.roles, a.specs, a.T = _p(roles), _p(specs_dev), len(specs)
    a.nodes, a.hi, a.P_total = _p(fb.nodes), _p(hi), P
    binvals = binvals.contiguous()
    exact = exact.contiguous()
    a.binvals, a.exact = _p(binvals), _p(exact)
    L.step(a, 9)
    reduce(hi, "min")
    L.step(a, 10)
    if L.gpu:
        torch.cuda.current_stream(dev).synchronize()   # keep the argument tensors alive
