"""Tables too large for HBM as float32: tree models train on streamed, binned-only data.

DeviceData(binned_only=True) streams the host rows (numpy / np.memmap) in chunks through
pinned buffers and keeps only the uint8 bins on the device; the edges come from the same
row sample the resident path uses, so bins, trees and CV scores are identical."""
import os

import numpy as np
import pytest
import torch

from cs230_distributed_machine_learning_amd.data.device import DeviceData
from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates
from cs230_distributed_machine_learning_amd.search.grid import ParameterGrid


def _table(n, d, seed=0):
    rng = np.random.RandomState(seed)
    X = rng.randn(n, d).astype(np.float32)
    y = (X[:, 0] + 0.5 * X[:, 1] ** 2 + 0.3 * rng.randn(n) > 0.4).astype(int)
    return X, y


def _scores(dd, model, grid):
    res = run_candidates(dd, JobSpec(model, list(ParameterGrid(grid)), cv=3), range(len(list(ParameterGrid(grid)))))
    assert all(r.ok for r in res), [r.error for r in res]
    return [r.result["cv_scores"] for r in res]


def _check(dev, n, d, chunk, tmp_path):
    X, y = _table(n, d)
    mm = np.lib.format.open_memmap(str(tmp_path / "X.npy"), mode="w+", dtype=np.float32, shape=X.shape)
    mm[:] = X
    mm.flush()
    Xmm = np.load(str(tmp_path / "X.npy"), mmap_mode="r")       # rows read from disk chunk by chunk
    res_dd = DeviceData(X, y, True, dev)
    bin_dd = DeviceData(Xmm, y, True, dev, binned_only=True, chunk_rows=chunk)
    assert bin_dd.X is None
    assert torch.equal(res_dd.edges.cpu(), bin_dd.edges.cpu())
    assert torch.equal(res_dd.binned().cpu(), bin_dd.binned().cpu())
    for model, grid in (("RandomForestClassifier", {"n_estimators": [8], "max_depth": [4, None]}),
                        ("GradientBoostingClassifier", {"n_estimators": [5], "max_depth": [2]})):
        assert _scores(res_dd, model, grid) == _scores(bin_dd, model, grid)
    # KNN: query blocks of held-out rows against streamed candidate chunks, exact merge
    knn_grid = {"n_neighbors": [1, 5, 12], "weights": ["uniform", "distance"], "p": [1, 2]}
    old_q = os.environ.get("DML_KNN_QBLOCK_GB")
    os.environ["DML_KNN_QBLOCK_GB"] = str(700 * d * 4 / 1e9)     # several query blocks
    try:
        assert _scores(res_dd, "KNeighborsClassifier", knn_grid) == _scores(bin_dd, "KNeighborsClassifier", knn_grid)
    finally:
        if old_q is None:
            os.environ.pop("DML_KNN_QBLOCK_GB")
        else:
            os.environ["DML_KNN_QBLOCK_GB"] = old_q
    # LogisticRegression streams the host rows once per objective evaluation (every candidate
    # x fold of the batch per chunk); the resident comparison runs the same fp32 objective
    lr_grid = {"C": [0.05, 1.0], "solver": ["lbfgs"], "max_iter": [200]}
    old = os.environ.get("DML_LR_MFMA")
    os.environ["DML_LR_MFMA"] = "0"
    try:
        a = _scores(res_dd, "LogisticRegression", lr_grid)
    finally:
        if old is None:
            os.environ.pop("DML_LR_MFMA")
        else:
            os.environ["DML_LR_MFMA"] = old
    np.testing.assert_allclose(np.asarray(_scores(bin_dd, "LogisticRegression", lr_grid)), np.asarray(a),
                               rtol=0, atol=1e-6)
    # LinearRegression / PCA re-stream the host rows for their moments and test rows
    rng = np.random.RandomState(1)
    yr = X @ rng.randn(d).astype(np.float32) + 3.0 + 0.1 * rng.randn(n).astype(np.float32)
    res_r = DeviceData(X, yr, False, dev)
    bin_r = DeviceData(Xmm, yr, False, dev, binned_only=True, chunk_rows=chunk)
    assert bin_r.X is None and bin_r.can_stream_rows()
    for model, grid in (("LinearRegression", {"fit_intercept": [True, False]}),
                        ("PCA", {"n_components": [2, 5]})):
        a, b = _scores(res_r, model, grid), _scores(bin_r, model, grid)
        np.testing.assert_allclose(np.asarray(b), np.asarray(a), rtol=1e-6, atol=1e-6)


def test_binned_only_svm_trains_on_host_rows(tmp_path):
    """SVC / SVR on a binned-only table: the host SMO on the table's host rows (the reference
    trains them on any table that fits in RAM), the same CV scores as a resident CPU table."""
    X, y = _table(1200, 6, seed=3)
    mm = np.lib.format.open_memmap(str(tmp_path / "X.npy"), mode="w+", dtype=np.float32, shape=X.shape)
    mm[:] = X
    mm.flush()
    Xmm = np.load(str(tmp_path / "X.npy"), mmap_mode="r")
    yr = (X[:, 0] * 2 + X[:, 1]).astype(np.float32)
    for clf, model, yy in ((True, "SVC", y), (False, "SVR", yr)):
        res = DeviceData(X, yy, clf, "cpu")
        binned = DeviceData(Xmm, yy, clf, "cpu", binned_only=True, chunk_rows=500)
        grid = {"C": [0.5, 2.0]}
        assert _scores(binned, model, grid) == _scores(res, model, grid)
    with pytest.raises(ValueError, match="binned form"):   # no host rows (bins received from a peer)
        nohost = DeviceData(Xmm, y, True, "cpu", binned_only=True)
        nohost._X_host = None
        run_candidates(nohost, JobSpec("SVC", [{"C": 1.0}], cv=3), [0])


def test_binned_only_cpu_matches_resident(tmp_path):
    _check("cpu", 5000, 9, 1234, tmp_path)


@pytest.mark.gpu
def test_binned_only_gpu_streaming_matches_resident(tmp_path):
    # > 200k rows: the edge sample path; small chunks: the pinned double-buffer pipeline
    _check("cuda:0", 260_000, 17, 50_000, tmp_path)


def _bcast_rank(rank, world, port, q):
    import os

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), OMP_NUM_THREADS="1")
    from cs230_distributed_machine_learning_amd.parallel import data as pdata
    from cs230_distributed_machine_learning_amd.parallel import dist

    dist.init(want_gpu=False, timeout_s=120)
    try:
        X, y = _table(3000, 7, seed=5) if rank == 0 else (None, None)
        dd = pdata.broadcast_binned(X, y, True, torch.device("cpu"), name="t")
        q.put((rank, dd.binned().numpy().copy(), dd.edges.numpy().copy(), list(dd.y_host[:20]),
               _scores(dd, "RandomForestClassifier", {"n_estimators": [6], "max_depth": [3, None]})))
    finally:
        dist.destroy()


def test_broadcast_binned_two_ranks_gloo():
    """The cluster runner's binned-only load: rank 0 bins, one broadcast of the bins."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_bcast_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict((r[0], r[1:]) for r in (q.get(timeout=180) for _ in range(2)))
    for p in ps:
        p.join(timeout=60)
    X, y = _table(3000, 7, seed=5)
    ref = DeviceData(X, y, True, "cpu")
    for r in (0, 1):
        Xb, E, y20, sc = out[r]
        assert np.array_equal(Xb, ref.binned().numpy()) and np.array_equal(E, ref.edges.numpy())
        assert list(y20) == list(y[:20])
    assert out[0][3] == out[1][3]


def test_stream_rows_covers_every_row_once():
    X, y = _table(1000, 5)
    dd = DeviceData(X, y, True, "cpu", binned_only=True, chunk_rows=300)
    got = [(r0, r1, xc.numpy()) for r0, r1, xc in dd.stream_rows()]
    assert [(a, b) for a, b, _ in got] == [(0, 300), (300, 600), (600, 900), (900, 1000)]
    assert np.array_equal(np.concatenate([x for _, _, x in got]), X)
    assert [(a, b) for a, b, _ in dd.stream_rows(5000)] == [(0, 1000)]
    res = DeviceData(X, y, True, "cpu")
    assert not res.can_stream_rows()
    with pytest.raises(ValueError):
        next(res.stream_rows())
