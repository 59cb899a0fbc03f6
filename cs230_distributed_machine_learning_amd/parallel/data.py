"""Dataset distribution across ranks (RCCL over xGMI), once per dataset.

Reference: every worker re-reads the full CSV from NFS/EFS for every task
(aws-prod/worker/worker.py:406-425; SURVEY §2.5 "the dominant data movement").  Here:

* ``broadcast_table`` — rank 0 parses the file once; its rows go host -> HBM -> every
  rank in 256 MB chunks, the H2D copy of chunk k overlapping the RCCL broadcast of chunk
  k-1 (``_pipelined_broadcast``); the table then
  stays resident across every candidate and job (``DeviceCache``).
* ``allgather_table`` — each rank holds a contiguous row shard (e.g. generated on the
  device, data/synthetic.py) and one ``all_gather_into_tensor`` assembles the table.
The uint8 binned copy is derived on each rank from edges broadcast by rank 0, so all
ranks grow identical trees for identical seeds.
"""
from __future__ import annotations

import json
import os
import threading
from typing import Callable, Dict, Optional, Set, Tuple

import numpy as np
import torch

from ..engine import faults
from . import dist


def broadcast_table(X: Optional[np.ndarray], y: Optional[np.ndarray], device: torch.device, y_kind: str = "auto",
                    group=None, tag: str = ""):
    """Rank 0 passes host arrays; every rank returns (X_dev, y_host_numpy).  ``group`` /
    ``tag``: the communicator and a key suffix unique to this load (concurrent loads on
    the runner's side group)."""
    inf = dist.info()
    st = dist.store()
    if not inf.is_dist:
        return torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32)).to(device), np.asarray(y)
    key = "dataset/meta" + tag
    if inf.rank == 0:
        y = np.asarray(y)
        # labels may be strings: ship a compact code array + the class table via the store
        if y.dtype.kind in "OUS":
            classes, codes = np.unique(y.astype(str), return_inverse=True)
            meta = {"n": int(X.shape[0]), "d": int(X.shape[1]), "y": "codes", "classes": classes.tolist()}
            y_num = codes.astype(np.float64)
        else:
            meta = {"n": int(X.shape[0]), "d": int(X.shape[1]), "y": str(y.dtype)}
            y_num = y.astype(np.float64)
        st.set(key, json.dumps(meta))
        yd = torch.from_numpy(y_num).to(device)
    else:
        st.wait([key])
        meta = json.loads(st.get(key))
        yd = None
    # every rank allocates its receive buffers, then all vote: a rank out of memory makes
    # EVERY rank give the load up before the broadcast (CollectiveAborted), instead of
    # leaving its peers inside a collective it never joins
    Xd, err = None, None
    try:
        faults.maybe_oom_in_collective(inf.rank, "load")
        if yd is None:
            yd = torch.empty((meta["n"],), dtype=torch.float64, device=device)
        Xd = torch.empty((meta["n"], meta["d"]), dtype=torch.float32, device=device)
    except torch.cuda.OutOfMemoryError as e:
        err = e
    except faults.InjectedOOM as e:
        err = e
    if not dist.vote_all_ok(err is None, group=group):
        Xd = yd = None
        if inf.rank == 0:
            st.delete_key(key)
        raise dist.CollectiveAborted(f"table load given up on every rank: a rank could not allocate "
                                     f"its {meta['n']}x{meta['d']} buffer" + (f" ({err})" if err else ""))
    _pipelined_broadcast(X if inf.rank == 0 else None, Xd, group=group)
    dist.broadcast(yd, 0, group=group)
    dist.barrier(group=group)
    if inf.rank == 0:
        st.delete_key(key)
        return Xd, y
    y_host = yd.cpu().numpy()
    if meta["y"] == "codes":
        y_host = np.asarray(meta["classes"], dtype=object)[y_host.astype(np.int64)]
    else:
        y_host = y_host.astype(np.dtype(meta["y"]))
    return Xd, y_host


BCAST_CHUNK_BYTES = 256 << 20


def _pipelined_broadcast(X: Optional[np.ndarray], Xd: torch.Tensor, chunk_bytes: Optional[int] = None,
                         group=None) -> None:
    """Root's host rows -> every rank's ``Xd``, in row chunks, H2D and broadcast overlapped.

    Rank 0 copies chunk k host -> HBM on a side stream (the pageable copy path runs at
    ~55 GB/s on MI355X, measured: profiles/r2_bcast_bench.log; staging through our own
    pinned buffers was slower, 25 GB/s, bound by the host memcpy) while RCCL broadcasts
    chunk k-1 over xGMI; the broadcast of a chunk waits only on that chunk's copy event.
    A single ``.to(device)`` followed by one broadcast would serialise the two.  The other
    ranks post one broadcast per chunk straight into their slice of ``Xd``."""
    n, d = Xd.shape
    if n == 0 or d == 0:
        return
    rows = max(1, (chunk_bytes or BCAST_CHUNK_BYTES) // (4 * d))
    root = dist.info().rank == 0
    gpu = Xd.is_cuda
    if root and gpu:
        copy_stream = torch.cuda.Stream(Xd.device)
        compute = torch.cuda.current_stream(Xd.device)
    for r0 in range(0, n, rows):
        r1 = min(n, r0 + rows)
        if root:
            src = torch.from_numpy(np.ascontiguousarray(X[r0:r1], dtype=np.float32))
            if gpu:
                with torch.cuda.stream(copy_stream):
                    Xd[r0:r1].copy_(src)
                    ev = torch.cuda.Event()
                    ev.record(copy_stream)
                compute.wait_event(ev)             # this chunk's broadcast follows its copy only
            else:
                Xd[r0:r1].copy_(src)
        dist.broadcast(Xd[r0:r1], 0, group=group)


def broadcast_binned(X: Optional[np.ndarray], y: Optional[np.ndarray], classification: bool, device: torch.device,
                     name: str = "", group=None, tag: str = ""):
    """Binned-only distribution of a table too large for HBM as float32 (tree jobs):
    rank 0 streams its host rows through the binning kernel (DeviceData binned_only),
    then ONE RCCL broadcast of the uint8 bins (+ edges) lands them on every rank -- a
    quarter of the float32 bytes over xGMI, and no rank ever holds the float32 table."""
    from ..data.device import DeviceData

    inf = dist.info()
    if not inf.is_dist:
        return DeviceData(X, y, classification, device, name=name, binned_only=True)
    st = dist.store()
    key = "dataset/binmeta" + tag
    if inf.rank == 0:
        _, y_host = broadcast_table(np.zeros((len(y), 0), dtype=np.float32), y, device, group=group, tag=tag)
        dd = DeviceData(X, y_host, classification, device, name=name, binned_only=True)
        buf, edges, smax = dd._Xb_full.contiguous(), dd._edges.contiguous(), dd._sample_max.contiguous().float()
        st.set(key, json.dumps({"n": int(buf.shape[0]), "ld": int(buf.shape[1]), "d": int(dd.d)}))
    else:
        _, y_host = broadcast_table(None, None, device, group=group, tag=tag)
        st.wait([key])
        meta = json.loads(st.get(key))
        buf = torch.empty((meta["n"], meta["ld"]), dtype=torch.uint8, device=device)
        edges = torch.empty((meta["d"], 255), dtype=torch.float32, device=device)
        smax = torch.empty((meta["d"],), dtype=torch.float32, device=device)
    dist.broadcast(buf, 0, group=group)
    dist.broadcast(edges, 0, group=group)
    dist.broadcast(smax, 0, group=group)
    dist.barrier(group=group)
    if inf.rank == 0:
        st.delete_key(key)
        return dd
    return DeviceData.from_bins(buf, meta["d"], edges, smax, y_host, classification, device, name=name)


def allgather_table(X_shard: torch.Tensor, y_shard: torch.Tensor):
    return dist.all_gather_rows(X_shard), dist.all_gather_rows(y_shard)


def share_bins(dd, group=None) -> None:
    """Rank 0 computes quantile edges; all ranks bin with the same edges."""
    from ..ops import binning

    inf = dist.info()
    if inf.rank == 0 or not inf.is_dist:
        edges = binning.quantile_edges(dd.X)
    else:
        edges = torch.empty((dd.d, binning.MAX_EDGES), dtype=torch.float32, device=dd.X.device)
    dist.broadcast(edges, 0, group=group)
    dd._edges = edges
    dd._Xb = binning.bin_matrix(dd.X, edges)


# ---- host-staged transport (no collective) ------------------------------------------------
# Used when a collective over the whole process group is impossible or not wanted: a rank
# died (the default group can no longer broadcast), or a worker joined after launch (it is
# not in the process group at all).  Rank 0 parses the table once and writes it to a
# host file (tmpfs by default); every rank memory-maps it and copies it to its own GPU over
# its own PCIe link -- no rank waits for another.
def _y_path(path: str) -> str:
    return path + ".y.npz"


_STAGE_LOCK = threading.Lock()
_STAGE_PATH_LOCKS: Dict[str, threading.Lock] = {}
_STAGE_PINNED: Set[str] = set()


def _path_lock(path: str) -> threading.Lock:
    with _STAGE_LOCK:
        return _STAGE_PATH_LOCKS.setdefault(path, threading.Lock())


def ensure_staged(load: Callable[[], Tuple[np.ndarray, np.ndarray]], path: str, pin: bool = False) -> str:
    """Stage the table at ``path`` exactly once per process, whichever thread asks first
    (rank 0's staging thread for host-staged jobs, its collective thread for sharded loads):
    a per-path lock makes a second caller wait for the first one's file instead of
    truncating it under a reader.  ``load()`` is called only when the file is missing.
    ``pin``: a host-staged job reads the file; ``release_staged`` keeps pinned files."""
    with _path_lock(path):
        if pin:
            _STAGE_PINNED.add(path)
        if not os.path.exists(path):
            X, y = load()
            stage_host(X, y, path)
    return path


def release_staged(path: str) -> bool:
    """Delete a staged table no host-staged job reads (a sharded load's transient copy in
    ``/dev/shm`` is host RAM on top of the registry's parsed copy)."""
    with _path_lock(path):
        if path in _STAGE_PINNED:
            return False
        for p in (path, _y_path(path)):
            try:
                os.remove(p)
            except OSError:
                pass
        return True


def stage_host(X: np.ndarray, y: np.ndarray, path: str, threads: int = 8) -> str:
    """Write the table for host-staged / sharded loads: X as a raw ``.npy`` (memory-mappable:
    a rank reads only the rows it copies) filled by ``threads`` parallel row-chunk copies
    (numpy releases the GIL for them), y + label metadata in a small sidecar.  Temporary
    names are unique per process and thread, and the final names appear by atomic rename."""
    from concurrent.futures import ThreadPoolExecutor

    y = np.asarray(y)
    meta = {"n": int(X.shape[0]), "d": int(X.shape[1])}
    if y.dtype.kind in "OUS":
        classes, codes = np.unique(y.astype(str), return_inverse=True)
        meta.update(y="codes", classes=classes.tolist())
        y_arr = codes.astype(np.int64)
    else:
        meta["y"] = str(y.dtype)
        y_arr = y
    uniq = f"{os.getpid()}.{threading.get_ident()}"
    tmp = f"{path}.{uniq}.tmp.npy"
    mm = np.lib.format.open_memmap(tmp, mode="w+", dtype=np.float32, shape=tuple(X.shape))
    n = X.shape[0]
    step = max(1, -(-n // max(1, threads * 4)))

    def copy(r0):
        mm[r0:r0 + step] = X[r0:r0 + step]

    with ThreadPoolExecutor(max_workers=max(1, threads)) as ex:
        list(ex.map(copy, range(0, n, step)))
    mm.flush()
    del mm
    ytmp = f"{_y_path(path)}.{uniq}.tmp.npz"
    np.savez(ytmp, y=y_arr, meta=np.array(json.dumps(meta)))
    os.replace(ytmp, _y_path(path))   # the sidecar first: a reader that sees X sees its labels
    os.replace(tmp, path)
    return path


def _staged_labels(path: str):
    with np.load(_y_path(path), allow_pickle=False) as z:
        meta = json.loads(str(z["meta"]))
        y = z["y"]
    if meta["y"] == "codes":
        y = np.asarray(meta["classes"], dtype=object)[y.astype(np.int64)]
    else:
        y = y.astype(np.dtype(meta["y"]))
    return meta, y


def _mapped_rows(Xm, device) -> torch.Tensor:
    """Rows of a read-only memory map on ``device``: a device copy straight from the mapped
    pages, or (CPU) a private writable copy -- never a tensor aliasing the read-only map."""
    import warnings

    dev = torch.device(device)
    if dev.type == "cpu":
        return torch.from_numpy(np.array(Xm, dtype=np.float32))
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", UserWarning)   # read-only source of a copy: nothing writes it
        return torch.from_numpy(np.asarray(Xm)).to(dev)


def load_staged(path: str, device: torch.device):
    """(X on ``device``, y host array) from a file written by ``stage_host``."""
    _, y = _staged_labels(path)
    return _mapped_rows(np.load(path, mmap_mode="r", allow_pickle=False), device), y


def sharded_load(path: str, device: torch.device, group=None):
    """Every rank of the group assembles the staged table: each copies ONLY its 1/N row block
    from the memory-mapped host file to its own GPU (N PCIe links in parallel instead of rank
    0's one), then one ``all_gather_into_tensor`` over xGMI (gloo: all_gather) completes the
    table on every rank.  Returns (X on ``device``, y host array, H2D seconds of
    this rank's block)."""
    import time

    inf = dist.info()
    meta, y = _staged_labels(path)
    n, d = meta["n"], meta["d"]
    Xm = np.load(path, mmap_mode="r", allow_pickle=False)
    if not inf.is_dist or inf.world == 1:
        t0 = time.perf_counter()
        X = _mapped_rows(Xm, device)
        return X, y, time.perf_counter() - t0
    W = inf.world
    q = -(-n // W)                                   # equal blocks (the last one padded)
    r0, r1 = min(n, inf.rank * q), min(n, (inf.rank + 1) * q)
    shard = full = None
    try:   # both buffers first, then a vote: an OOM on one rank aborts the load on every rank
        faults.maybe_oom_in_collective(inf.rank, "load")
        shard = torch.zeros((q, d), dtype=torch.float32, device=device)
        full = torch.empty((W * q, d), dtype=torch.float32, device=device)
        ok = True
    except (torch.cuda.OutOfMemoryError, faults.InjectedOOM):
        ok = False
    if not dist.vote_all_ok(ok, group=group):
        shard = full = None
        raise dist.CollectiveAborted(f"sharded load given up on every rank: a rank could not allocate {n}x{d}")
    t0 = time.perf_counter()
    if r1 > r0:
        shard[:r1 - r0].copy_(_mapped_rows(Xm[r0:r1], device))
    if shard.is_cuda:
        torch.cuda.synchronize(device)
    h2d = time.perf_counter() - t0
    full = dist.all_gather_rows(shard, group=group, out=full)   # [W * q, d] in rank order
    dist.barrier(group=group)
    return full[:n], y, h2d
