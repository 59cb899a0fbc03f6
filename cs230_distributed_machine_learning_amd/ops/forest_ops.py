"""Batched forest build / predict / score on GPU (HIP) or CPU (C++).

The GPU entry points drive ``libdml_hip.so`` (csrc/kernels/forest.hip, predict.hip);
the CPU ones drive ``libdml_cpu.so`` (csrc/runtime/forest_cpu.cpp).  Both consume the
same ``TREESPEC_DTYPE`` records and produce the same pool layout:

* ``nodes``  int32 [P, 2] — (feature*256 + bin | -1, left child | -1); right = left+1
* ``vals``   float64 [P, VC] — class weight sums (classification) or (sum w, sum wy,
  sum wy^2) (regression)
* tree ``t`` of the batch has its root at node ``t``.
"""
from __future__ import annotations

import ctypes
import os
import sys
import math
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch

from ..utils import native
from ..utils import trace

GINI, ENTROPY, MSE, POISSON, MAE, FRIEDMAN = 0, 1, 2, 3, 4, 5   # MAE: build_cpu / build_gpu_mae
INT32_MAX = 2**31 - 1


@dataclass
class ForestTiers:
    """Node-size tiers of the HIP builder (see forest.hip header)."""

    sub_max: int = 64          # <= 64 rows: one wave finishes the whole subtree (k_subtree)
    sub_small: int = 32        # subtree roots of <= 32 rows: tier 4, half-size LDS row cache (2x per CU)
    sub_cache_max_d: int = 256  # cache the subtree's bin rows in LDS when d <= this
    wave_max: int = 512         # sweeps: profiles/r1_forest_ab_experiments.md, r2_tier_sweep.txt
    # binary classification (2-wave block-tier nodes, forest.hip DML_BLOCK_NT): the block tier
    # takes nodes above 256 rows -- sweep build 0.974 -> 0.960 s (profiles/r6_block_nt128_sweep.txt)
    wave_max_bin: int = 256
    block_max: int = 65536      # r5 (block tier at 4 WGs/CU): 65536 vs 32768 -1.7 % sweep build, bench +2.6 %
                                # (profiles/r5_block_max_sweep.txt; r2 kernels: 32768 beat 131072 by 4 %)
    chunk: int = 16384
    # builds whose trees all evaluate every feature (boosting, max_features=None) whose
    # whole-feature large-tier histograms fit DML_LARGE_SUB_GB: nodes above this many rows take
    # the large tier, where the larger of two siblings is derived from the parent's histogram
    # (GBRT config 6: 6.38 -> 7.32 CV-fits/s at 2048, 7.17 at 8192, 7.27 at 1024)
    block_max_all: int = 2048
    kg_wave: int = 4
    kg_block: int = 16
    kg_large: int = 16
    # regression builds (boosting stages): smaller large-tier row chunks and feature rounds,
    # i.e. more, smaller workgroups in flight (several per CU) -- config 6 repeated sweep:
    # 13.7 (16384-row chunks) -> 14.9 (8192) -> 15.4 CV-fits/s (4096);
    # profiles/r4_gbrt_cfg6_chunk_sweep.txt
    chunk_reg: int = 4096
    kg_large_reg: int = 16
    slack_wave: int = 0
    # binary classification, > 0: nodes of sub_max < count <= bigsub_max grow their WHOLE
    # subtree in one 4-wave workgroup from an LDS row cache (forest.hip k_bigsub) and tier 1
    # is capped at it.  Off by default: 1.605 vs 1.050 s on the sweep build (the 25.6 KB row
    # cache allows 3 workgroups per CU, each mostly one busy wave; nodes of 257..512 rows move
    # to the block tier) -- profiles/r4_bigsub.md
    bigsub_max: int = 0

    def fitted(self, n_channels: int) -> "ForestTiers":
        """Clamp feature-group sizes to the LDS budget for this channel count."""
        per_feat = n_channels * 256 * 4
        t = ForestTiers(**self.__dict__)
        for k in t.__dict__:   # experiments: DML_TIER_<FIELD>=<int> overrides a field
            env = os.environ.get("DML_TIER_" + k.upper())
            if env:
                setattr(t, k, int(env))
        if n_channels == 3 and not os.environ.get("DML_TIER_WAVE_MAX"):   # binary classification
            t.wave_max = min(t.wave_max, t.wave_max_bin)
        t.kg_wave = max(1, min(t.kg_wave, (24 * 1024) // per_feat, 4))     # k_nodes<64>: KGMAX 4
        t.kg_block = max(1, min(t.kg_block, (96 * 1024) // per_feat, 16))  # k_nodes<256>: KGMAX 16
        t.kg_large = max(1, min(t.kg_large, (96 * 1024) // per_feat, 64))
        t.kg_large_reg = max(1, min(t.kg_large_reg, (96 * 1024) // per_feat, 64))
        return t


@dataclass
class ForestBuild:
    nodes: object  # torch.Tensor (cuda) or np.ndarray
    vals: object
    n_trees: int
    VC: int
    is_reg: bool
    n_classes: int
    stats: dict = field(default_factory=dict)

    @property
    def on_gpu(self) -> bool:
        return isinstance(self.nodes, torch.Tensor) and self.nodes.is_cuda

    def to_numpy(self) -> "ForestBuild":
        if isinstance(self.nodes, torch.Tensor):
            return ForestBuild(self.nodes.cpu().numpy(), self.vals.cpu().numpy(), self.n_trees, self.VC,
                               self.is_reg, self.n_classes, dict(self.stats))
        return self


def _sub_cache_stride(d: int) -> int:
    """Row stride (bytes) of the subtree LDS cache: multiple of 4 with an odd word count
    so 32 lanes reading the same feature hit 32 distinct banks."""
    dp = (d + 3) // 4 * 4
    if (dp // 4) % 2 == 0:
        dp += 4
    return dp


def make_specs(n: int) -> np.ndarray:
    return np.zeros(n, dtype=native.TREESPEC_DTYPE)


def _pool_bound(counts: np.ndarray, specs: np.ndarray) -> int:
    msl = np.maximum(specs["min_samples_leaf"].astype(np.int64), 1)
    leaves = np.maximum(counts // msl, 1)
    depth = specs["max_depth"].astype(np.int64)
    depth_cap = np.where(depth < 40, (np.int64(2) ** np.minimum(depth + 1, 40)) - 1, np.int64(2**62))
    per = np.minimum(2 * leaves + 1, depth_cap)
    return int(per.sum()) + 16


class _Arena:
    """Per-device byte buffers reused by successive forest builds (grow-only).

    A forest batch needs a workspace and a node pool of tens of GB whose sizes change
    from batch to batch; fresh ``torch.empty`` calls of that size miss the caching
    allocator and fall through to hipMalloc / release-and-retry, which measured ~1.1 s
    per batch (a third of the bench step).  The arena keeps one buffer per slot and
    device, grown with 50% headroom (capped by free HBM) when a batch needs more, and hands out views.
    Slot ``"forest"`` holds a build's workspace AND node pool and stays taken until the
    caller's ``release_pool`` (the forest family, which is done with a batch's trees
    before the next build; ``ForestFamily.presize`` sizes it once per job).  Slot
    ``"ws"`` is a workspace-only slot for builds whose trees outlive the call (boosting)."""

    def __init__(self):
        self.bufs: Dict[tuple, torch.Tensor] = {}
        self.busy: set = set()
        self.grows: List[tuple] = []   # (slot, old bytes, new bytes, seconds) of every mid-run regrowth
        self.lock = threading.Lock()

    def take(self, dev: torch.device, slot: str, nbytes: int) -> Optional[torch.Tensor]:
        key = (dev.index if dev.index is not None else torch.cuda.current_device(), slot)
        with self.lock:
            if key in self.busy:
                if os.environ.get("DML_ARENA_LOG"):
                    print(f"[arena] {slot} busy: fresh allocation of {nbytes / 1e9:.2f} GB", file=sys.stderr, flush=True)
                return None              # another build on this device holds it: allocate fresh
            buf = self.bufs.get(key)
            if buf is None or buf.numel() < nbytes:
                t_grow = time.perf_counter()
                old = 0 if buf is None else int(buf.numel())
                self.bufs.pop(key, None)
                del buf
                # grow with 50% headroom (batch sizes vary; every regrowth is a slow
                # hipMalloc), but never past 70% of what the device can still give (kernel scratch and
                # runtime queues need the rest: a 0.8 budget fraction ran the queue out of resources)
                free, _ = torch.cuda.mem_get_info(dev)
                spare = free + torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
                target = max(int(nbytes), min(int(nbytes * 3 // 2), int(0.7 * spare)))
                buf = torch.empty(target, dtype=torch.uint8, device=dev)
                self.bufs[key] = buf
                self.grows.append((slot, old, target, time.perf_counter() - t_grow))
                if os.environ.get("DML_ARENA_LOG"):
                    print(f"[arena] grow {slot}: {old / 1e9:.2f} -> {target / 1e9:.2f} GB (need {nbytes / 1e9:.2f}) "
                          f"{self.grows[-1][3]:.3f}s", file=sys.stderr, flush=True)
            self.busy.add(key)
            return buf

    def reserve(self, dev: torch.device, slot: str, nbytes: int) -> int:
        """Grow an idle slot to ``nbytes`` now (job setup), so the batches of the job never
        regrow it mid-run (each regrowth is a multi-GB hipMalloc).  Capped at 70% of
        what the device can still give; returns the slot's size."""
        key = (dev.index if dev.index is not None else torch.cuda.current_device(), slot)
        with self.lock:
            if key in self.busy:
                return 0
            buf = self.bufs.get(key)
            if buf is not None and buf.numel() >= nbytes:
                return int(buf.numel())
            if buf is not None:
                self.bufs.pop(key)
                del buf
                torch.cuda.empty_cache()
            free, _ = torch.cuda.mem_get_info(dev)
            spare = free + torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
            target = int(min(int(nbytes), int(0.7 * spare)))
            self.bufs[key] = torch.empty(target, dtype=torch.uint8, device=dev)
            return target

    def give(self, dev: torch.device, slot: str) -> None:
        key = (dev.index if dev.index is not None else torch.cuda.current_device(), slot)
        with self.lock:
            self.busy.discard(key)

    def clear(self, dev: torch.device) -> None:
        """Return the idle slots of ``dev`` to the device (another family needs the HBM)."""
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        with self.lock:
            drop = [k for k in self.bufs if k[0] == idx and k not in self.busy]
            for k in drop:
                del self.bufs[k]
        if drop:
            torch.cuda.empty_cache()
        # the builder's own whole-histogram buffers (forest.hip FullBufs, outside this arena)
        with torch.cuda.device(dev):
            native.hip_lib().dml_forest_release_scratch()

    def held_bytes(self, dev: torch.device) -> int:
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        with self.lock:
            return sum(int(b.numel()) for (i, _s), b in self.bufs.items() if i == idx and (i, _s) not in self.busy)


ARENA = _Arena()


def workspace_bytes(rows_total: int, T: int, d: int, n_classes: int, is_reg: bool,
                    tiers: "ForestTiers | None" = None) -> int:
    """Device workspace of a build with ``rows_total`` active rows over ``T`` trees
    (the C++ planner's own layout, csrc/kernels/forest.hip ``plan``)."""
    CH = 4 if is_reg else n_classes + 1
    t = (tiers or ForestTiers()).fitted(CH)
    a = native.ForestArgs()
    a.d, a.n_classes, a.is_reg, a.T = d, (n_classes if not is_reg else 1), int(is_reg), T
    a.rows_total = int(rows_total)
    a.wave_max, a.block_max, a.chunk = t.wave_max, t.block_max, t.chunk
    a.kg_wave, a.kg_block, a.kg_large, a.slack_wave, a.sub_max = t.kg_wave, t.kg_block, t.kg_large, t.slack_wave, t.sub_max
    a.sub_small = t.sub_small
    if _bigsub_on(t, is_reg, n_classes, d, None):   # the smaller tier 1 has more block-tier nodes
        a.wave_max = min(t.wave_max, t.bigsub_max)
    return int(native.hip_lib().dml_forest_workspace_bytes(ctypes.byref(a)))


def _bigsub_on(t: "ForestTiers", is_reg: bool, n_classes: int, d: int, mono) -> bool:
    """The big-subtree tier applies: binary classification, no monotonic constraints, the
    subtree row cache on (forest.hip k_bigsub; DML_BIGSUB=0 turns it off)."""
    return (t.bigsub_max > t.sub_max and not is_reg and n_classes == 2 and mono is None
            and d <= t.sub_cache_max_d and os.environ.get("DML_BIGSUB", "1") != "0")


TOP_SLOTS_MAX = 256   # room per tree for predict.hip's top table (kTopSlots = 1 << kTopLv <= 256)


def pool_bytes(pool_cap: int, VC: int) -> int:
    return (pool_cap * 8 + 255) // 256 * 256 + pool_cap * VC * 8


def _carve(buf: torch.Tensor, off: int, shape, dtype) -> torch.Tensor:
    n = int(np.prod(shape)) * torch.tensor([], dtype=dtype).element_size()
    return buf[off:off + n].view(dtype).view(*shape)


EXP_OFF, EXP_BINS = 160, 320   # bucket k + EXP_OFF of a target's frexp exponent k (|y| < 2^k)


_LANE = threading.local()


def set_build_lane(lane: int) -> None:
    """Select the calling thread's build lane (forest.hip ``dml_forest_set_lane``): concurrent
    builds from different host threads need different lanes -- each lane has its own side
    streams, read-back words, whole-histogram buffers and workspace arena slot."""
    if native.hip_lib().dml_forest_set_lane(int(lane)) < 0:
        raise ValueError(f"build lane {lane} out of range")
    _LANE.v = int(lane)


def build_lane() -> int:
    return getattr(_LANE, "v", 0)


def _h2d(arr: np.ndarray, dev) -> torch.Tensor:
    """Host array -> device without a host/GPU rendezvous: staged through pinned memory and
    copied on the stream (a pageable copy blocks the host until the stream has drained, so the
    GPU sits idle while the host prepares the next launches).  The caching host allocator keeps
    the pinned staging buffer alive until the copy has run."""
    t = torch.from_numpy(np.ascontiguousarray(arr))
    if dev.type != "cuda":
        return t.to(dev)
    return t.pin_memory().to(dev, non_blocking=True)


def reg_exponent_counts(yreg, n: int, ystride: int = 0, targets: int = 1, defer: bool = False):
    """Per-target histogram of the frexp exponents of the nonzero targets: int64
    [targets, EXP_BINS] (a torch tensor on ``yreg``'s device, or numpy).  Counts are exact
    and order-free, so every builder -- and every rank of a row-sharded build, after a sum
    all-reduce -- derives the same exponents from them (``reg_exponents_of_counts``).
    ``ystride > 0``: target t is ``yreg[t * ystride : t * ystride + n]``.
    ``defer`` (device path): return a callable that checks and returns the counts, so the
    caller can read them back with its own next host/GPU sync."""
    targets = max(1, int(targets)) if ystride > 0 else 1
    if torch.is_tensor(yreg) and yreg.is_cuda and yreg.dtype == torch.float32 and yreg.is_contiguous():
        # one LDS-histogram kernel (gbrt.hip k_exp_hist): boosting recounts every stage's targets
        lib = native.hip_lib()
        cnt = torch.zeros((targets, EXP_BINS), dtype=torch.int64, device=yreg.device)
        bad = torch.zeros(1, dtype=torch.int64, device=yreg.device)
        rc = lib.dml_exp_hist(native.ptr(yreg), n, ystride if ystride > 0 else n, targets, native.ptr(cnt),
                              native.ptr(bad), native.stream_handle(yreg.device))
        if rc != 0:
            raise RuntimeError(f"dml_exp_hist failed ({rc})")

        def resolve():
            if int(bad.item()):
                raise ValueError("regression target contains NaN or infinity")
            return cnt

        return resolve if defer else resolve()
    if torch.is_tensor(yreg):
        y = yreg.reshape(-1)
        rows = y[: (targets - 1) * ystride + n].as_strided((targets, n), (ystride, 1)) if ystride > 0 else y[:n][None]
        if not bool(torch.isfinite(rows).all()):
            raise ValueError("regression target contains NaN or infinity")
        k = torch.frexp(rows.float())[1].to(torch.int64) + EXP_OFF
        k = torch.where(rows != 0, k, torch.zeros_like(k))          # bucket 0: zeros (never a float32 exponent)
        k += torch.arange(targets, device=k.device, dtype=torch.int64)[:, None] * EXP_BINS
        cnt = torch.zeros(targets * EXP_BINS, dtype=torch.int64, device=k.device)
        cnt.scatter_add_(0, k.reshape(-1), torch.ones_like(k).reshape(-1))
        return cnt.view(targets, EXP_BINS)
    y = np.asarray(yreg, dtype=np.float32).reshape(-1)
    rows = (np.lib.stride_tricks.as_strided(y, (targets, n), (ystride * 4, 4)) if ystride > 0 else y[None, :n])
    if not np.isfinite(rows).all():
        raise ValueError("regression target contains NaN or infinity")
    k = np.frexp(rows)[1].astype(np.int64) + EXP_OFF
    k[rows == 0] = 0
    cnt = np.zeros((targets, EXP_BINS), dtype=np.int64)
    for t in range(targets):
        cnt[t] = np.bincount(k[t], minlength=EXP_BINS)
    return cnt


def _max_exponent(cnt):
    """k such that every target of the exponent histogram has |y| < 2^k (None: all zero)."""
    c = np.asarray(cnt.cpu() if torch.is_tensor(cnt) else cnt, dtype=np.int64).reshape(-1, EXP_BINS)
    nz = np.nonzero(c[:, 1:].any(axis=0))[0]
    return int(nz[-1] + 1 - EXP_OFF) if len(nz) else None


def reg_exponents_of_counts(cnt) -> tuple[int, int]:
    """The fixed-point rule (forest_common.h ``reg_exponents_counts`` is the same loop):
    B1 = max over targets of sum_k c_k 2^k >= sum |y|, B2 likewise with 4^k >= sum y^2;
    e1 = 61 - ceil-exponent(15 B1), e2 from 15 B2 -- so any bootstrap-weighted (w <= 15)
    sum over a tree's rows stays below 2^61 in magnitude.  The y^2 grid is therefore set
    by the target's total energy, not by n max|y|^2: a node of small targets next to a few
    huge ones keeps its variance (review finding: one outlier used to zero every small
    node's y^2 and turn it into a pure leaf).  Exact counts summed in fixed k order: the
    HIP, the C++ and the row-sharded builders agree bit for bit."""
    c = np.asarray(cnt.cpu() if torch.is_tensor(cnt) else cnt, dtype=np.int64).reshape(-1, EXP_BINS)
    k = np.arange(EXP_BINS, dtype=np.float64) - EXP_OFF
    c = c.astype(np.float64)
    c[:, 0] = 0.0                                   # bucket 0 holds the zeros
    # cumsum is a strictly sequential float64 sum in bucket order (the C loop's order);
    # every term c_k 2^k is exact
    b1 = float(np.cumsum(c * np.ldexp(1.0, k.astype(np.int64)), axis=1)[:, -1].max())
    b2 = float(np.cumsum(c * np.ldexp(1.0, 2 * k.astype(np.int64)), axis=1)[:, -1].max())
    clamp = lambda e: max(-1000, min(1000, e))
    e1 = clamp(61 - math.frexp(15.0 * b1)[1]) if b1 > 0 else 0
    e2 = clamp(61 - math.frexp(15.0 * b2)[1]) if b2 > 0 else 0
    return e1, e2


def reg_exponents(yreg, n: int, ystride: int = 0, targets: int = 1) -> tuple[int, int]:
    """Fixed-point exponents (e1, e2) of a regression build (``reg_exponents_of_counts``
    of the targets' exponent histogram)."""
    if yreg is None or n <= 0:
        return 0, 0
    return reg_exponents_of_counts(reg_exponent_counts(yreg, n, ystride, targets))


def _n_targets(specs: np.ndarray, ystride: int) -> int:
    return int(specs["target"].max()) + 1 if ystride > 0 and len(specs) else 1


def build_gpu_mae(Xb: torch.Tensor, yreg: torch.Tensor, roles: torch.Tensor, specs: np.ndarray) -> ForestBuild:
    """criterion="absolute_error" regression trees on the GPU (csrc/kernels/forest_mae.hip):
    rows kept in (y, row id) order, exact fixed-point abs deviations -- the host builder's
    trees node for node.  ``yreg`` float32 [n] on the device."""
    lib = native.hip_lib()
    dev = Xb.device
    n, d = Xb.shape
    T = len(specs)
    y = yreg.float().contiguous()
    specs_dev = torch.from_numpy(specs.view(np.uint8).copy()).to(dev)
    e1, e2 = reg_exponents(y, n)
    perm = torch.sort(y, stable=True).indices.to(torch.int32).contiguous()   # (y, row id) order
    counts = torch.zeros(T, dtype=torch.int32, device=dev)
    a = native.MaeArgs()
    a.Xb, a.ld, a.n, a.d = native.ptr(Xb), Xb.stride(0), n, d
    a.yreg, a.roles, a.specs, a.T, a.perm = native.ptr(y), native.ptr(roles), native.ptr(specs_dev), T, native.ptr(perm)
    a.yq_e1, a.yq_e2, a.counts = e1, e2, native.ptr(counts)
    stream = native.stream_handle(dev)
    t0 = time.perf_counter()
    with trace.range("forest_count"):
        if lib.dml_mae_count(ctypes.byref(a), stream):
            raise RuntimeError(f"dml_mae_count failed: {native.hip_error(lib)}")
        cnt = counts.cpu().numpy().astype(np.int64)
    row_off = np.zeros(T + 1, dtype=np.int64)
    np.cumsum(cnt, out=row_off[1:])
    row_off_dev = torch.from_numpy(row_off).to(dev)
    pool_cap = _pool_bound(cnt, specs) + T
    rows_a = torch.empty(max(1, int(row_off[-1])), dtype=torch.int32, device=dev)
    rows_b = torch.empty_like(rows_a)
    nodes = torch.empty((pool_cap, 2), dtype=torch.int32, device=dev)
    vals = torch.empty((pool_cap, 3), dtype=torch.float64, device=dev)
    nabs = torch.empty(pool_cap, dtype=torch.float64, device=dev)
    osz = int(lib.dml_mae_sizeof_open())
    open_a = torch.empty(pool_cap * osz, dtype=torch.uint8, device=dev)
    open_b = torch.empty_like(open_a)
    counters = torch.zeros(8, dtype=torch.int32, device=dev)
    tree_W = torch.empty(T, dtype=torch.float64, device=dev)
    # nodes of >= big_rows rows evaluate their first P visiting positions on one workgroup
    # each (a level holds at most rows / big_rows + T of them)
    big_rows = max(256, int(os.environ.get("DML_MAE_BIG_ROWS", "8192")))
    P = int(min(d, int(specs["max_features"].max()) + 2)) if T else 1
    big_cap = int(row_off[-1]) // big_rows + T + 1
    big_a = torch.empty(big_cap * osz, dtype=torch.uint8, device=dev)
    big_b = torch.empty_like(big_a)
    res = torch.empty(big_cap * P * int(lib.dml_mae_sizeof_res()), dtype=torch.uint8, device=dev)
    a.big_a, a.big_b, a.big_cap = native.ptr(big_a), native.ptr(big_b), big_cap
    a.res, a.P, a.big_rows = native.ptr(res), P, big_rows
    a.row_off, a.rows_a, a.rows_b = native.ptr(row_off_dev), native.ptr(rows_a), native.ptr(rows_b)
    a.nodes, a.vals, a.nabs, a.pool_cap = native.ptr(nodes), native.ptr(vals), native.ptr(nabs), pool_cap
    a.open_a, a.open_b, a.open_cap = native.ptr(open_a), native.ptr(open_b), pool_cap
    a.counters, a.tree_W = native.ptr(counters), native.ptr(tree_W)
    with trace.range("forest_build"):
        if lib.dml_mae_build(ctypes.byref(a), stream):
            raise RuntimeError(f"dml_mae_build failed: {native.hip_error(lib)}")
    if a.status_out:
        raise RuntimeError(f"dml_mae_build status {a.status_out} (1: node pool overflow)")
    P = int(a.n_nodes_out)
    return ForestBuild(nodes[:P], vals[:P], T, 3, True, 1,
                       stats={"levels": int(a.levels_out), "nodes": P, "build_s": time.perf_counter() - t0,
                              "builder": "gpu-mae"})


def build_gpu(Xb: torch.Tensor, ycls: Optional[torch.Tensor], yreg: Optional[torch.Tensor], roles: torch.Tensor,
              specs: np.ndarray, n_classes: int, is_reg: bool, tiers: ForestTiers | None = None,
              ystride: int = 0, reuse_pool: bool = False, XbT: Optional[torch.Tensor] = None,
              cw: Optional[np.ndarray] = None, mono: Optional[np.ndarray] = None,
              early_predict=None, count_cache: Optional[dict] = None,
              root_counts: Optional[dict] = None) -> ForestBuild:
    """``ystride > 0``: ``yreg`` is a [targets, ystride] matrix and tree t regresses on
    row ``specs[t]['target']`` (gradient boosting's per-fit pseudo-residuals).
    ``reuse_pool``: the node arrays live in the device arena and are valid until the
    next ``reuse_pool`` build on this device (the caller must be done with them).
    ``early_predict``: (make(nodes, vals) -> GpuPredict, done int32[F]) -- fit f is predicted
    by the builder right after level done[f] (its trees are complete by then), overlapping the
    deeper fits; entries it launched come back as -2 (``ForestBuild.predict`` holds the
    GpuPredict; the caller predicts the other fits).
    ``count_cache``: a dict kept by the caller for as long as ``roles`` and the specs' split /
    bootstrap fields stay the same (boosting stages of one active set): the per-tree active-row
    counts are computed once into it and reused (no count kernel, no read-back).
    ``root_counts`` (boosting, same lifetime as ``count_cache``): a dict holding a uint32
    [T, d, 256] device cache of the trees' root-histogram row counts; the first build fills it
    (``valid`` becomes 1), later builds skip the root level's count atomics and copy them in."""
    lib = native.hip_lib()
    dev = Xb.device
    T = len(specs)
    n, d = Xb.shape
    CH = 4 if is_reg else n_classes + 1
    VC = 3 if is_reg else n_classes
    tiers = (tiers or ForestTiers()).fitted(CH)
    stream = native.stream_handle(dev)
    specs_dev = _h2d(specs.view(np.uint8), dev)
    cached = count_cache is not None and "active" in count_cache
    active = count_cache["active"] if cached else torch.zeros(T, dtype=torch.int32, device=dev)
    a = native.ForestArgs()
    a.Xb, a.ld, a.n, a.d = native.ptr(Xb), Xb.stride(0), n, d
    a.ycls = native.ptr(ycls) if ycls is not None else 0
    a.yreg = native.ptr(yreg) if yreg is not None else 0
    a.n_classes, a.is_reg = (n_classes if not is_reg else 1), int(is_reg)
    # the targets' exponent histogram is launched here and read back together with the
    # active-row counts below (one host/GPU sync for both)
    exp_cnt = (reg_exponent_counts(yreg, n, ystride, _n_targets(specs, ystride), defer=True)
               if is_reg and yreg is not None and n > 0 else None)
    a.yq_e1, a.yq_e2 = 0, 0
    a.roles, a.n_splits = native.ptr(roles), roles.shape[0]
    a.specs, a.T = native.ptr(specs_dev), T
    a.ystride = int(ystride)
    if XbT is not None:
        assert XbT.shape == (d, n) and XbT.dtype == torch.uint8 and XbT.is_contiguous() and XbT.device == dev
    a.XbT = native.ptr(XbT) if XbT is not None else 0
    # class-weight table [T, C] float64 (rows of cw_mode 2 trees are filled by the kernel)
    cw_dev = None
    if cw is not None and not is_reg:
        cw_dev = _h2d(np.ascontiguousarray(cw, dtype=np.float64).reshape(T, n_classes), dev)
    a.cw = native.ptr(cw_dev) if cw_dev is not None else 0
    # monotonic_cst: int8 [fits][d] rows indexed by the specs' "fit" (classifier rows
    # constrain the class-0 fraction, i.e. arrive negated) + per-node bounds
    mono_dev = None
    if mono is not None and np.any(mono):
        mono_dev = _h2d(np.ascontiguousarray(mono, dtype=np.int8), dev)
    a.mono = native.ptr(mono_dev) if mono_dev is not None else 0
    a.nbound = 0
    # one criterion, no class weights / monotonic constraints / min_weight_fraction_leaf: the
    # HIP node kernels specialised on that criterion run (forest.hip spec_of / specialise)
    crits = np.unique(specs["criterion"]) if T else np.zeros(0)
    if (T and set(crits.tolist()) <= {MSE, FRIEDMAN} and FRIEDMAN in crits
            and not np.any(specs["min_impurity_decrease"] > 0)):
        # friedman_mse ranks splits exactly like squared_error (forest_common.h); only the
        # min_impurity_decrease test differs, and with none set the squared-error kernels grow
        # the same trees (gradient boosting's default criterion)
        crits = np.array([MSE])
    a.fast_crit = (int(crits[0]) + 1 if len(crits) == 1 and cw_dev is None and mono_dev is None
                   and not np.any(specs["min_weight_frac"] > 0) else 0)
    a.active_count = native.ptr(active)
    # every tree unit-weight (no bootstrap, e.g. boosting stages): compact large-tier LDS slices
    a.large_unit = int(bool(is_reg and T and np.all(specs["bootstrap"] == 0)))
    if root_counts is not None and is_reg and T:
        buf = root_counts.get("buf")
        if buf is None or buf.numel() != T * d * 256:
            buf = root_counts["buf"] = torch.empty(T * d * 256, dtype=torch.int32, device=dev)
            root_counts["valid"] = 0
        a.root_counts, a.root_counts_valid = native.ptr(buf), int(root_counts.get("valid", 0))
    t0 = time.perf_counter()
    with trace.range("forest_count"):
        if cached:
            counts, row_off, row_off_dev = count_cache["counts"], count_cache["row_off"], count_cache["row_off_dev"]
        else:
            rc = lib.dml_forest_count(ctypes.byref(a), stream)
            if rc:
                raise RuntimeError(f"dml_forest_count failed ({rc}): {native.hip_error(lib)}")
            counts = active.cpu().numpy().astype(np.int64)
    kmax = None   # |y| < 2^kmax for every target of the build (exponent histogram)
    if exp_cnt is not None:
        cnt = exp_cnt() if callable(exp_cnt) else exp_cnt
        a.yq_e1, a.yq_e2 = reg_exponents_of_counts(cnt)
        kmax = _max_exponent(cnt)
    if not cached:
        row_off = np.zeros(T + 1, dtype=np.int64)
        np.cumsum(counts, out=row_off[1:])
        row_off_dev = _h2d(row_off, dev)
        if count_cache is not None:
            count_cache.update(active=active, counts=counts, row_off=row_off, row_off_dev=row_off_dev)
    a.row_off = native.ptr(row_off_dev)
    a.rows_total = int(row_off[-1])
    a.max_active = int(counts.max()) if T else 0
    pool_cap = _pool_bound(counts, specs) + T
    a.wave_max, a.block_max, a.chunk = tiers.wave_max, tiers.block_max, (tiers.chunk_reg if is_reg else tiers.chunk)
    a.kg_wave, a.kg_block, a.slack_wave = tiers.kg_wave, tiers.kg_block, tiers.slack_wave
    if T and os.environ.get("DML_TIER_KG_BLOCK") is None:
        # block tier: feature groups no wider than the batch's largest max_features (a node's
        # first group is min(kg_block, max_features) features either way, so no tree changes):
        # the LDS histogram slab shrinks with it (max_features=10: 22 KB instead of 34 KB,
        # 7 instead of 4 block-tier nodes per CU)
        a.kg_block = max(1, min(int(a.kg_block), int(min(d, int(specs["max_features"].max())))))
    a.kg_large = tiers.kg_large_reg if is_reg else tiers.kg_large
    # unit-weight regression build whose fixed-point targets stay below 2^39 in magnitude:
    # the large tier packs each row's count and w yq into ONE u64 LDS atomic (forest.hip
    # kPackShift; <= 4095 rows per workgroup) -- the count atomic was ~3/4 of the histogram
    # time below the boosting root (profiles/r5_gbrt_root_hist_micro.txt)
    a.large_pack = 0
    if (is_reg and a.large_unit and kmax is not None and kmax + int(a.yq_e1) <= 38
            and os.environ.get("DML_LARGE_NO_PACK", "0") == "0"):
        a.large_pack = 1
        a.chunk = min(int(a.chunk), 3840)
    if is_reg and d > 0:
        # whole-feature regression rounds of equal width (100 features: 7 rounds of 15 / 10,
        # not 6 of 16 and one of 4) -- GBRT config 6 16.7 -> 17.1 CV-fits/s,
        # profiles/r5_gbrt_cfg6_kg_sweep_compact.txt
        a.kg_large = -(-d // -(-d // int(a.kg_large)))
    a.sub_max = tiers.sub_max
    a.sub_small = tiers.sub_small
    a.sub_cache_d = _sub_cache_stride(d) if d <= tiers.sub_cache_max_d else 0
    a.all_features = int(T > 0 and bool(np.all(specs["max_features"] >= d)))
    if a.all_features and 0 < tiers.block_max_all < a.block_max:
        depth = int(min(30, specs["max_depth"].max()))
        per_level = T * min(a.max_active // tiers.block_max_all + 1, 1 << depth)
        node_b = d * 256 * (2 * 8 if is_reg else (n_classes + 1) * 4)   # forest.hip ghist_feat_bytes
        if per_level * node_b <= float(os.environ.get("DML_LARGE_SUB_GB", "4")) * 1e9:
            a.block_max = tiers.block_max_all
    big = _bigsub_on(tiers, is_reg, n_classes, d, mono_dev) and a.sub_cache_d > 0
    a.bigsub_max = min(tiers.bigsub_max, 256) if big else 0
    if big:
        a.wave_max = min(tiers.wave_max, a.bigsub_max)
    tree_W = torch.empty(T, dtype=torch.float64, device=dev)
    a.tree_W = native.ptr(tree_W)
    ws_bytes = lib.dml_forest_workspace_bytes(ctypes.byref(a))
    ws_span = (ws_bytes + 255) // 256 * 256
    # reuse_pool (the forest family): workspace and node pool share ONE arena slot,
    # "forest", held until release_pool -- any batch under the family's HBM budget fits
    # the presized slot whatever its split between rows (workspace) and nodes (pool).
    # Otherwise (boosting keeps its trees): arena workspace + freshly allocated pool.
    slot = None
    ws_buf = None
    ws_slot = "ws" if build_lane() == 0 else f"ws{build_lane()}"   # one workspace per lane
    if not reuse_pool:
        with trace.range("forest_alloc"):
            ws_buf = ARENA.take(dev, ws_slot, ws_bytes)
            workspace = ws_buf[:ws_bytes] if ws_buf is not None else torch.empty(ws_bytes, dtype=torch.uint8,
                                                                                  device=dev)
    retries = 0
    try:
        for _attempt in range(4):
            with trace.range("forest_alloc"):
                vals_off = (pool_cap * 8 + 255) // 256 * 256
                pbytes = pool_bytes(pool_cap, VC)
                if reuse_pool:
                    if slot is not None:               # a pool retry needs a bigger slot
                        ARENA.give(dev, slot)
                        slot = None
                    buf = ARENA.take(dev, "forest", ws_span + pbytes)
                    if buf is not None:
                        slot = "forest"
                    else:
                        buf = torch.empty(ws_span + pbytes, dtype=torch.uint8, device=dev)
                    workspace = buf[:ws_bytes]
                    nodes = _carve(buf, ws_span, (pool_cap, 2), torch.int32)
                    vals = _carve(buf, ws_span + vals_off, (pool_cap, VC), torch.float64)
                else:
                    nodes = torch.empty((pool_cap, 2), dtype=torch.int32, device=dev)
                    vals = torch.empty((pool_cap, VC), dtype=torch.float64, device=dev)
            a.workspace, a.workspace_bytes = native.ptr(workspace), ws_bytes
            a.nodes, a.node_val, a.pool_cap = native.ptr(nodes), native.ptr(vals), pool_cap
            if mono_dev is not None:   # every pool slot starts unbounded
                nbound = torch.empty((pool_cap, 2), dtype=torch.float64, device=dev)
                nbound[:, 0] = -math.inf
                nbound[:, 1] = math.inf
                a.nbound = native.ptr(nbound)
            a.status_out = 0
            gp = None
            if early_predict is not None:   # (re)armed per attempt: a pool retry regrows from scratch
                make, done = early_predict
                if _attempt == 0:
                    done0 = done.copy()
                done[:] = done0
                gp = make(nodes, vals)
                a.early_pred, a.fit_done_level, a.n_fits = ctypes.addressof(gp.args), done.ctypes.data, len(done)
            with trace.range("forest_build"):   # host-side launch sequence of every tier
                rc = lib.dml_forest_build(ctypes.byref(a), stream)
            if rc:
                raise RuntimeError(f"dml_forest_build failed ({rc}): {native.hip_error(lib)}")
            if a.status_out == 1:
                pool_cap *= 2
                retries += 1
                continue
            if a.status_out != 0:
                raise RuntimeError(f"dml_forest_build status {a.status_out}")
            break
        else:
            raise RuntimeError("forest node pool overflow")
    except BaseException:
        if slot is not None:
            ARENA.give(dev, slot)
        raise
    finally:
        # stream order keeps the next build's kernels behind this build's on the same stream
        if ws_buf is not None:
            ARENA.give(dev, ws_slot)
    if root_counts is not None and a.root_counts:
        root_counts["valid"] = int(a.root_counts_valid)
    P = int(a.n_nodes_out)
    del workspace
    stats = {"levels": int(a.levels_out), "large_rounds": int(a.large_rounds_out), "nodes": P,
             "rows_total": int(a.rows_total), "build_s": time.perf_counter() - t0, "pool_retries": retries,
             "tier_nodes": [int(a.tier0_nodes), int(a.tier1_nodes), int(a.tier2_nodes), int(a.tier3_nodes)]}
    fb = ForestBuild(nodes[:P], vals[:P], T, VC, is_reg, n_classes, stats)
    if early_predict is not None:
        fb.predict = gp
        fb.early_done = early_predict[1]
    if slot is not None:
        fb.arena_dev = dev   # release_pool(fb) hands the arena slot back
        fb.arena_slot = slot
    return fb


def release_pool(fb: ForestBuild) -> None:
    """The caller is done with a ``reuse_pool`` build's node arrays."""
    dev = getattr(fb, "arena_dev", None)
    if dev is not None:
        fb.nodes = fb.vals = None
        fb.arena_dev = None
        ARENA.give(dev, getattr(fb, "arena_slot", "forest"))


def build_cpu(Xb: np.ndarray, ycls: Optional[np.ndarray], yreg: Optional[np.ndarray], roles: np.ndarray,
              specs: np.ndarray, n_classes: int, is_reg: bool, ystride: int = 0,
              cw: Optional[np.ndarray] = None, mono: Optional[np.ndarray] = None) -> ForestBuild:
    """The C++ host builder.  ``mono``: int8 [fits, d] monotonic constraints indexed by
    the specs' ``fit`` (classifier rows constrain the class-0 fraction), or None."""
    lib = native.cpu_lib()
    Xb = np.ascontiguousarray(Xb, dtype=np.uint8)
    roles = np.ascontiguousarray(roles, dtype=np.uint8)
    specs = np.ascontiguousarray(specs)
    ycls = None if ycls is None else np.ascontiguousarray(ycls, dtype=np.int32)
    yreg = None if yreg is None else np.ascontiguousarray(yreg, dtype=np.float32)
    n, d = Xb.shape
    T = len(specs)
    VC = 3 if is_reg else n_classes
    t0 = time.perf_counter()
    cw = None if (cw is None or is_reg) else np.ascontiguousarray(cw, dtype=np.float64).reshape(T, n_classes)
    mono = None if mono is None else np.ascontiguousarray(mono, dtype=np.int8)
    e1, e2 = reg_exponents(yreg, n, ystride, _n_targets(specs, ystride)) if is_reg else (0, 0)
    h = lib.dml_cpu_forest_build_mono(native.ptr(Xb), d, n, d, native.ptr(ycls), native.ptr(yreg),
                                      (1 if is_reg else n_classes), int(is_reg), native.ptr(roles), native.ptr(specs),
                                      T, int(ystride), native.ptr(cw), native.ptr(mono), e1, e2)
    try:
        P = lib.dml_cpu_forest_num_nodes(h)
        nodes = np.empty((P, 2), dtype=np.int32)
        vals = np.empty((P, VC), dtype=np.float64)
        lib.dml_cpu_forest_export(h, native.ptr(nodes), native.ptr(vals))
    finally:
        lib.dml_cpu_forest_free(h)
    return ForestBuild(nodes, vals, T, VC, is_reg, n_classes, {"nodes": int(P), "build_s": time.perf_counter() - t0})


PRUNE_SCRATCH_BYTES = 256 << 20


def prune_max_leaves(fb: ForestBuild, specs: np.ndarray, limit: np.ndarray) -> np.ndarray:
    """max_leaf_nodes: keep each limited tree's best-first top (sklearn's
    BestFirstTreeBuilder order; csrc/kernels/forest_common.h best_first_prune), in place.
    ``limit``: int32 [T], 0 = unlimited.  Returns the leaf count per tree (-1 = untouched)."""
    T = len(specs)
    limit = np.ascontiguousarray(limit, dtype=np.int32)
    lim_trees = np.nonzero(limit > 0)[0]
    if lim_trees.size == 0:
        return np.full(T, -1, dtype=np.int32)
    VC, C = int(fb.VC), (1 if fb.is_reg else int(fb.n_classes))
    if not fb.on_gpu:
        leaves = np.empty(T, dtype=np.int32)
        specs_c = np.ascontiguousarray(specs)
        native.cpu_lib().dml_cpu_forest_prune(native.ptr(fb.nodes), native.ptr(fb.vals), VC, C, int(fb.is_reg),
                                              native.ptr(specs_c), native.ptr(limit), T, native.ptr(leaves))
        return leaves
    dev = fb.nodes.device
    lib = native.hip_lib()
    specs_dev = torch.from_numpy(specs.view(np.uint8).copy()).to(dev)
    lim_dev = torch.from_numpy(limit).to(dev)
    leaves = torch.full((T,), -1, dtype=torch.int32, device=dev)
    cap = int(limit.max())
    per = max(1, PRUNE_SCRATCH_BYTES // (16 * cap))
    t, t_end = int(lim_trees[0]), int(lim_trees[-1]) + 1
    heap = torch.empty(min(per, t_end - t) * cap * 16, dtype=torch.uint8, device=dev)
    stream = native.stream_handle(dev)
    while t < t_end:
        n = min(per, t_end - t)
        rc = lib.dml_forest_prune(native.ptr(fb.nodes), native.ptr(fb.vals), VC, C, int(fb.is_reg),
                                  native.ptr(specs_dev), native.ptr(lim_dev), t, n, native.ptr(heap), cap,
                                  native.ptr(leaves), stream)
        if rc:
            raise RuntimeError(f"dml_forest_prune failed ({rc})")
        t += n
    return leaves.cpu().numpy()   # also keeps specs_dev / heap alive until the kernels are done


def prune_ccp(fb: ForestBuild, specs: np.ndarray, alpha: np.ndarray) -> np.ndarray:
    """Minimal cost-complexity pruning (sklearn ``ccp_alpha``), in place, on the device.

    sklearn prunes the weakest link (smallest effective alpha
    ``g(t) = (R(t) - R(T_t)) / (|leaves(T_t)| - 1)``) while ``g <= ccp_alpha``, with
    ``R(t) = W_t / W_root * impurity(t)``.  That sequence ends in the smallest subtree
    minimising ``R(T) + alpha * |leaves(T)|`` (Breiman et al.), which is one bottom-up
    pass: a node becomes a leaf when ``R(t) + alpha <= the best cost of its subtree``.
    The pass runs level by level from the leaves up, vectorised over every tree of the
    batch (breadth-first levels of the pool, as ``extract_forest`` walks them).
    ``alpha``: float64 [T] (0 = leave the tree alone).  Returns leaves per tree."""
    T = len(specs)
    on_np = not isinstance(fb.nodes, torch.Tensor)
    nodes = torch.from_numpy(fb.nodes) if on_np else fb.nodes
    vals = torch.from_numpy(fb.vals) if on_np else fb.vals
    dev = nodes.device
    a = torch.from_numpy(np.ascontiguousarray(alpha, dtype=np.float64)).to(dev)
    crit = torch.from_numpy(np.ascontiguousarray(specs["criterion"], dtype=np.int64)).to(dev)
    v = vals.double()
    if fb.is_reg:
        w = v[:, 0]
        m = v[:, 1] / w.clamp_min(1e-300)
        imp = torch.where(w > 0, v[:, 2] / w.clamp_min(1e-300) - m * m, torch.zeros_like(w))
    else:
        w = v.sum(1)
        p = v / w.clamp_min(1e-300).unsqueeze(1)
        gini = 1.0 - (p * p).sum(1)
        ent = -(torch.where(p > 0, p * torch.log2(p.clamp_min(1e-300)), torch.zeros_like(p))).sum(1)
    levels = []
    fo = torch.arange(T, dtype=torch.int64, device=dev)
    tr = fo.clone()
    while fo.numel():
        levels.append((fo, tr))
        rec = nodes[fo]
        internal = rec[:, 0] >= 0
        l = rec[internal, 1].to(torch.int64)
        tr = tr[internal].repeat_interleave(2)
        fo = torch.stack([l, l + 1], 1).reshape(-1)
    W_root = w[:T]
    cost = torch.zeros(nodes.shape[0], dtype=torch.float64, device=dev)
    leaves = torch.zeros(nodes.shape[0], dtype=torch.int64, device=dev)
    for fo, tr in reversed(levels):
        if fb.is_reg:
            im = imp[fo]
        else:
            im = torch.where(crit[tr] == ENTROPY, ent[fo], gini[fo])
        R = w[fo] / W_root[tr] * im
        leaf_cost = R + a[tr]
        rec = nodes[fo]
        internal = rec[:, 0] >= 0
        l = rec[:, 1].clamp_min(0).to(torch.int64)
        sub = torch.where(internal, cost[l] + cost[l + 1], leaf_cost)
        nl = torch.where(internal, leaves[l] + leaves[l + 1], torch.ones_like(l))
        cut = internal & (a[tr] > 0) & (leaf_cost <= sub)
        cost[fo] = torch.where(cut | ~internal, leaf_cost, sub)
        leaves[fo] = torch.where(cut, torch.ones_like(nl), nl)
        if bool(cut.any()):
            idx = fo[cut]
            nodes[idx] = torch.tensor([-1, -1], dtype=nodes.dtype, device=dev)
    return leaves[:T].cpu().numpy()


def refine_thresholds(fb: ForestBuild, Xb, specs: np.ndarray, roles, vals, exact) -> None:
    """Move split bins to sklearn's midpoint thresholds on exactly-binned features (in place)."""
    T = len(specs)
    P = int(fb.nodes.shape[0])
    if fb.on_gpu:
        dev = Xb.device
        specs_dev = torch.from_numpy(specs.view(np.uint8).copy()).to(dev)
        hi = torch.empty(P, dtype=torch.int32, device=dev)
        rc = native.hip_lib().dml_forest_refine(native.ptr(Xb), Xb.stride(0), Xb.shape[0], Xb.shape[1],
                                                native.ptr(fb.nodes), P,
                                                native.ptr(specs_dev), T, native.ptr(roles), native.ptr(vals),
                                                native.ptr(exact), native.ptr(hi), native.stream_handle(dev))
        if rc:
            raise RuntimeError("dml_forest_refine failed")
        torch.cuda.current_stream(dev).synchronize()   # keep specs_dev / hi alive until done
        return
    Xb_np = np.ascontiguousarray(Xb)
    roles_np = np.ascontiguousarray(roles, dtype=np.uint8)
    specs_c = np.ascontiguousarray(specs)
    native.cpu_lib().dml_cpu_forest_refine(native.ptr(Xb_np), Xb_np.shape[1], Xb_np.shape[0], native.ptr(fb.nodes), P,
                                           native.ptr(specs_c), T, native.ptr(roles_np), native.ptr(vals),
                                           native.ptr(exact))


def apply(fb: ForestBuild, Xb, t0: int = 0, T: Optional[int] = None):
    """Leaf node index of every row for trees t0..t0+T-1: int32 [T, n]."""
    T = fb.n_trees - t0 if T is None else T
    n = Xb.shape[0]
    if fb.on_gpu:
        leaf = torch.empty((T, n), dtype=torch.int32, device=Xb.device)
        rc = native.hip_lib().dml_forest_apply(native.ptr(Xb), Xb.stride(0), n, native.ptr(fb.nodes), t0, T,
                                               native.ptr(leaf), native.stream_handle(Xb.device))
        if rc:
            raise RuntimeError("dml_forest_apply failed")
        return leaf
    Xb = np.ascontiguousarray(Xb)
    nodes = np.ascontiguousarray(fb.nodes, dtype=np.int32)
    leaf = np.empty((T, n), dtype=np.int32)
    native.cpu_lib().dml_cpu_forest_apply(native.ptr(Xb), Xb.shape[1], n, native.ptr(nodes), t0, T, native.ptr(leaf))
    return leaf


class GpuPredict:
    """A GPU predict of F fits set up before (or after) their build: device offset arrays,
    output buffers and the ``PredictArgs`` block.  ``run(fits)`` predicts a subset of the
    fits (one launch each); the forest builder takes ``args`` and predicts a fit itself as
    soon as its trees are complete (ForestArgs.early_pred)."""

    def __init__(self, nodes, vals, VC: int, is_reg: bool, n_classes: int, Xb, fit_tree_off, fit_row_off, rows,
                 want_proba: bool = False, depth_cap=None):
        dev = Xb.device
        F = len(fit_tree_off) - 1
        total = int(fit_row_off[-1])
        C = n_classes
        self.dev, self.F = dev, F
        self.toff = torch.from_numpy(np.asarray(fit_tree_off, dtype=np.int32)).to(dev)
        self.roff_host = np.ascontiguousarray(fit_row_off, dtype=np.int64)
        self.roff = torch.from_numpy(self.roff_host).to(dev)
        self.rows = rows if isinstance(rows, torch.Tensor) else torch.from_numpy(np.asarray(rows, np.int32)).to(dev)
        self.out = torch.empty(total, dtype=torch.float32 if is_reg else torch.int32, device=dev)
        self.proba = torch.empty((total, C), dtype=torch.float32, device=dev) if (want_proba and not is_reg) else None
        p = native.PredictArgs()
        p.Xb, p.ld = native.ptr(Xb), Xb.stride(0)
        p.nodes, p.node_val, p.VC, p.is_reg, p.n_classes = native.ptr(nodes), native.ptr(vals), VC, int(is_reg), C
        p.fit_tree_off, p.fit_row_off, p.rows = native.ptr(self.toff), native.ptr(self.roff), native.ptr(self.rows)
        p.out_pred, p.out_proba = native.ptr(self.out), native.ptr(self.proba)
        p.F = F
        p.d = int(Xb.shape[1])
        p.max_rows = int(np.max(np.diff(self.roff_host))) if F else 0
        p.fit_row_off_host = self.roff_host.ctypes.data
        if depth_cap is not None:   # int32 [F]: fit f walks its trees down to this depth (<= 0: all)
            self._cap = torch.from_numpy(np.ascontiguousarray(depth_cap, dtype=np.int32)).to(dev)
            p.fit_depth_cap = native.ptr(self._cap)
        toff = np.asarray(fit_tree_off, dtype=np.int64)
        if F and int(toff[-1]) > 0:
            # every tree's first levels, heap-ordered (predict.hip k_top_fill), read by the walk
            # from LDS: up to TOP_SLOTS_MAX NodeRecs (8 B) per tree, indexed by tree id
            self._top = torch.empty((int(toff.max()) * TOP_SLOTS_MAX, 2), dtype=torch.int32, device=dev)
            p.toptab, p.max_trees = native.ptr(self._top), int(np.max(np.diff(toff)))
        self.args = p

    def run(self, fits=None) -> None:
        """Predict ``fits`` (None: all) in ONE launch (grid.y = fit; fits outside the list
        exit at once through the skip mask) -- the deep fits left after the build's early
        predicts run concurrently instead of one launch after another."""
        lib = native.hip_lib()
        st = native.stream_handle(self.dev)
        with trace.range("forest_predict"):
            if fits is not None and len(fits) == 0:
                return
            if fits is None or len(fits) == self.F:
                self.args.fit_skip = 0
                rc = lib.dml_forest_predict(ctypes.byref(self.args), st)
            elif len(fits) == 1:
                rc = lib.dml_forest_predict_fit(ctypes.byref(self.args), int(fits[0]), st)
            else:
                skip = np.ones(self.F, dtype=np.int32)
                skip[np.asarray(list(fits), dtype=np.int64)] = 0
                self._skip = torch.from_numpy(skip).to(self.dev, non_blocking=False)
                self.args.fit_skip = native.ptr(self._skip)
                rc = lib.dml_forest_predict(ctypes.byref(self.args), st)
                self.args.fit_skip = 0
        if rc:
            raise RuntimeError(f"dml_forest_predict failed ({rc})")

    def result(self):
        return (self.out, self.proba) if self.proba is not None else self.out


def predict(fb: ForestBuild, Xb, fit_tree_off: np.ndarray, fit_row_off: np.ndarray, rows, want_proba: bool = False,
            depth_cap=None):
    """Predict rows for F fits; trees of fit f are [fit_tree_off[f], fit_tree_off[f+1]) (GPU:
    read down to depth_cap[f] when given -- a max_depth prefix of deeper grown trees)."""
    F = len(fit_tree_off) - 1
    total = int(fit_row_off[-1])
    C = fb.n_classes
    if fb.on_gpu:
        gp = GpuPredict(fb.nodes, fb.vals, fb.VC, fb.is_reg, C, Xb, fit_tree_off, fit_row_off, rows, want_proba,
                        depth_cap=depth_cap)
        gp.run()
        out, proba = gp.out, gp.proba
        return (out, proba) if want_proba else out
    if depth_cap is not None and np.any(np.asarray(depth_cap) > 0):
        raise ValueError("depth-capped predict runs on the GPU predictor only")
    lib = native.cpu_lib()
    Xb = np.ascontiguousarray(Xb)
    rows_np = np.ascontiguousarray(rows, dtype=np.int32)
    toff = np.ascontiguousarray(fit_tree_off, dtype=np.int32)
    roff = np.ascontiguousarray(fit_row_off, dtype=np.int64)
    nodes = np.ascontiguousarray(fb.nodes, dtype=np.int32)
    vals = np.ascontiguousarray(fb.vals, dtype=np.float64)
    out_cls = np.empty(total, dtype=np.int32) if not fb.is_reg else None
    out_reg = np.empty(total, dtype=np.float32) if fb.is_reg else None
    proba = np.empty((total, C), dtype=np.float32) if (want_proba and not fb.is_reg) else None
    lib.dml_cpu_forest_predict(native.ptr(Xb), Xb.shape[1], native.ptr(nodes), native.ptr(vals), fb.VC, int(fb.is_reg), C,
                               native.ptr(toff), native.ptr(roff), native.ptr(rows_np), F, native.ptr(out_cls),
                               native.ptr(out_reg), native.ptr(proba))
    out = out_reg if fb.is_reg else out_cls
    return (out, proba) if want_proba else out


def score_stats(rows, fit_row_off: np.ndarray, pred, ycls=None, yreg=None, is_reg: bool = False) -> np.ndarray:
    """[F, 4] = (correct | SSE, sum y, sum y^2, n) per fit — fused K10 kernel on GPU."""
    F = len(fit_row_off) - 1
    if isinstance(pred, torch.Tensor) and pred.is_cuda:
        dev = pred.device
        out = torch.empty((F, 4), dtype=torch.float64, device=dev)
        roff = torch.from_numpy(np.asarray(fit_row_off, dtype=np.int64)).to(dev)
        s = native.ScoreArgs()
        s.rows, s.fit_row_off, s.pred = native.ptr(rows), native.ptr(roff), native.ptr(pred)
        s.ycls, s.yreg, s.is_reg = native.ptr(ycls), native.ptr(yreg), int(is_reg)
        s.out, s.F = native.ptr(out), F
        rc = native.hip_lib().dml_scores(ctypes.byref(s), native.stream_handle(dev))
        if rc:
            raise RuntimeError("dml_scores failed")
        return out.cpu().numpy()
    rows = np.asarray(rows)
    out = np.zeros((F, 4), dtype=np.float64)
    for f in range(F):
        r = rows[fit_row_off[f]:fit_row_off[f + 1]]
        p = np.asarray(pred)[fit_row_off[f]:fit_row_off[f + 1]]
        if is_reg:
            y = np.asarray(yreg)[r].astype(np.float64)
            out[f] = (np.sum((p.astype(np.float64) - y) ** 2), y.sum(), (y * y).sum(), len(r))
        else:
            out[f] = (np.sum(p == np.asarray(ycls)[r]), 0.0, 0.0, len(r))
    return out
