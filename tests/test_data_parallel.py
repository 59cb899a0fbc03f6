"""Row-sharded data-parallel fits (parallel/data_parallel.py) on CPU with gloo.

Every rank holds only its row block; the loss/gradient (LogisticRegression) and the
normal equations (LinearRegression) are all-reduced.  The CV scores must equal the
single-process fits of the full table, and every rank must agree."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from cs230_distributed_machine_learning_amd.parallel.data_parallel import shard_bounds

# row-sharded forests: per-level histogram all-reduce (ops/forest_dp.py)
RF_GRID = [{"n_estimators": 8, "max_depth": md, "min_samples_leaf": msl, "class_weight": cw, "random_state": 5}
           for md, msl, cw in ((None, 1, None), (6, 3, "balanced"), (None, 2, "balanced_subsample"))] + \
          [{"n_estimators": 6, "criterion": "entropy", "max_features": 0.5, "random_state": 2}]
KNN_GRID = [{"n_neighbors": k, "weights": w, "metric": m} for k, w, m in
            ((5, "uniform", "minkowski"), (9, "distance", "manhattan"), (3, "uniform", "chebyshev"))]
GB_GRID = [{"n_estimators": 12, "max_depth": 3, "learning_rate": 0.3, "random_state": 1},
           {"n_estimators": 8, "max_depth": 2, "subsample": 0.7, "random_state": 2}]
PCA_GRID = [{"n_components": k} for k in (2, 5, "mle")] + [{"n_components": 4, "whiten": True}]
RFR_GRID = [{"n_estimators": 5, "max_depth": 8, "random_state": 1}, {"n_estimators": 4, "min_samples_leaf": 5}]
LR_GRID = [{"C": c, "solver": s, "class_weight": cw, "max_iter": 200}
           for c in (0.05, 1.0) for s in ("liblinear", "newton-cg") for cw in (None, "balanced")]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _table(n=3001, d=12, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d)).astype(np.float32)
    w = rng.normal(size=d)
    z = X @ w + 0.7 * rng.normal(size=n)
    y_cls = np.digitize(z, [-1.0, 0.8])            # 3 unbalanced classes
    y_reg = (z + 0.1 * rng.normal(size=n)).astype(np.float64)
    return X, y_cls, y_reg


def _run(data_cls, X, y, model, cands, cv=4, **kw):
    from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates

    spec = JobSpec(model, cands, cv=cv, holdout=True, test_size=0.2, random_state=3, keep_models="none")
    res = run_candidates(data_cls, spec, range(len(cands)))
    assert all(r.ok for r in res), [r.error for r in res if not r.ok]
    return [(r.result["cv_scores"], r.result.get("accuracy", r.result.get("r2_score"))) for r in res]


def _rank(rank, world, port, outq):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), OMP_NUM_THREADS="2")
    try:
        from cs230_distributed_machine_learning_amd.parallel import dist
        from cs230_distributed_machine_learning_amd.parallel.data_parallel import RowShard, scatter_table

        from cs230_distributed_machine_learning_amd.parallel import data_parallel

        inf = dist.init(want_gpu=False, timeout_s=120)
        X, y_cls, y_reg = _table()
        # rows leave rank 0 in chunks (ADVICE: rank 0 must not hold every block): force
        # many small chunks so the chunk boundaries are exercised
        data_parallel.SCATTER_CHUNK_BYTES = 4 * X.shape[1] * 97
        Xs, yg, r0 = scatter_table(X if rank == 0 else None, y_cls if rank == 0 else None, inf.device)
        assert (r0, r0 + Xs.shape[0]) == shard_bounds(len(X), world, rank)
        assert np.array_equal(yg, y_cls) and np.allclose(Xs.numpy(), X[r0:r0 + Xs.shape[0]])
        # the replicated path: rank 0's rows broadcast in many pipelined chunks
        from cs230_distributed_machine_learning_amd.parallel import data as pdata

        pdata.BCAST_CHUNK_BYTES = 4 * X.shape[1] * 101
        Xf, yf = pdata.broadcast_table(X if rank == 0 else None, y_cls if rank == 0 else None, inf.device)
        assert np.array_equal(Xf.numpy(), X) and np.array_equal(np.asarray(yf), y_cls)
        sh = RowShard(Xs, yg, r0, True, inf.device)
        lr = _run(sh, X, yg, "LogisticRegression", LR_GRID)
        a, b = shard_bounds(len(X), world, rank)
        shr = RowShard(X[a:b], y_reg, a, False, inf.device)
        lin = _run(shr, X, y_reg, "LinearRegression", [{"fit_intercept": True}, {"fit_intercept": False}], cv=3)
        rf = _run(sh, X, yg, "RandomForestClassifier", RF_GRID, cv=3)
        rfr = _run(shr, X, y_reg, "RandomForestRegressor", RFR_GRID, cv=3)
        knn = _run(sh, X, yg, "KNeighborsClassifier", KNN_GRID, cv=3)
        knr = _run(shr, X, y_reg, "KNeighborsRegressor", KNN_GRID[:2], cv=3)
        err = None
        try:
            _run(sh, X, yg, "SVC", [{"C": 1.0}])
        except ValueError as e:
            err = str(e)
        pca = _run(shr, X, y_reg, "PCA", PCA_GRID, cv=3)
        gbc = _run(sh, X, yg, "GradientBoostingClassifier", GB_GRID, cv=3)
        gbr = _run(shr, X, y_reg, "GradientBoostingRegressor", GB_GRID[:1], cv=3)
        gb_err = None
        try:
            _run(shr, X, y_reg, "GradientBoostingRegressor", [{"loss": "huber", "n_estimators": 3}], cv=3)
        except AssertionError as e:
            gb_err = str(e)
        outq.put(("ok", rank, lr, lin, err, rf, rfr, knn, knr, pca, gbc, gbr, gb_err))
        dist.destroy()
    except Exception:  # pragma: no cover
        import traceback

        outq.put(("err", rank, traceback.format_exc()))


def test_row_sharded_fits_match_single_process():
    from cs230_distributed_machine_learning_amd.data.device import DeviceData

    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        outs = [q.get(timeout=600) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=120)
            if p.is_alive():
                p.kill()
    for o in outs:
        assert o[0] == "ok", o[2]
    X, y_cls, y_reg = _table()
    ref_lr = _run(DeviceData(X, y_cls, True), X, y_cls, "LogisticRegression", LR_GRID)
    ref_lin = _run(DeviceData(X, y_reg, False), X, y_reg, "LinearRegression",
                   [{"fit_intercept": True}, {"fit_intercept": False}], cv=3)
    o0, o1 = sorted(outs, key=lambda o: o[1])
    assert o0[2] == o1[2] and o0[3] == o1[3]           # every rank reports the same scores
    for (cv_s, hold), (cv_r, hold_r) in zip(o0[2], ref_lr):
        # float32 gradients summed in another order: identical up to a few near-tie rows
        assert np.allclose(cv_s, cv_r, atol=2.5e-3), (cv_s, cv_r)
        assert abs(hold - hold_r) <= 2.5e-3
    for (cv_s, hold), (cv_r, hold_r) in zip(o0[3], ref_lin):
        assert np.allclose(cv_s, cv_r, atol=1e-9) and abs(hold - hold_r) < 1e-9
    assert o0[4] and "row-sharded" in o0[4]
    # classification forests are the SAME forests the one-process builder grows (integer
    # histograms summed over ranks): identical scores; regression sums floats in another
    # order, so near-tie splits may differ
    ref_rf = _run(DeviceData(X, y_cls, True), X, y_cls, "RandomForestClassifier", RF_GRID, cv=3)
    assert o0[5] == o1[5] and o0[6] == o1[6]
    assert o0[5] == ref_rf, (o0[5], ref_rf)
    # row-sharded KNN: per-rank top-K + exact merge = the one-process neighbours
    assert o0[7] == o1[7] and o0[8] == o1[8]
    assert o0[7] == _run(DeviceData(X, y_cls, True), X, y_cls, "KNeighborsClassifier", KNN_GRID, cv=3)
    ref_knr = _run(DeviceData(X, y_reg, False), X, y_reg, "KNeighborsRegressor", KNN_GRID[:2], cv=3)
    for (cv_s, hold), (cv_r, hold_r) in zip(o0[8], ref_knr):
        assert np.allclose(cv_s, cv_r, atol=1e-9) and abs(hold - hold_r) < 1e-9
    # row-sharded PCA: all-reduced moments and held-out log-likelihood sums
    assert o0[9] == o1[9]
    ref_pca = _run(DeviceData(X, y_reg, False), X, y_reg, "PCA", PCA_GRID, cv=3)
    for (cv_s, hold), (cv_r, hold_r) in zip(o0[9], ref_pca):
        assert np.allclose(cv_s, cv_r, rtol=1e-9, atol=1e-9), (cv_s, cv_r)
    # row-sharded boosting: regression stage trees over fp32 histograms summed across ranks
    # (near-tie splits may differ), all-reduced Newton leaf sums, global subsample draws
    assert o0[10] == o1[10] and o0[11] == o1[11]
    ref_gbc = _run(DeviceData(X, y_cls, True), X, y_cls, "GradientBoostingClassifier", GB_GRID, cv=3)
    for (cv_s, hold), (cv_r, hold_r) in zip(o0[10], ref_gbc):
        assert np.allclose(cv_s, cv_r, atol=0.02) and abs(hold - hold_r) <= 0.02, (cv_s, cv_r)
    ref_gbr = _run(DeviceData(X, y_reg, False), X, y_reg, "GradientBoostingRegressor", GB_GRID[:1], cv=3)
    for (cv_s, hold), (cv_r, hold_r) in zip(o0[11], ref_gbr):
        assert np.allclose(cv_s, cv_r, atol=0.02) and abs(hold - hold_r) <= 0.02, (cv_s, cv_r)
    assert o0[12] and "row-sharded GradientBoosting" in o0[12]
    ref_rfr = _run(DeviceData(X, y_reg, False), X, y_reg, "RandomForestRegressor", RFR_GRID, cv=3)
    for (cv_s, hold), (cv_r, hold_r) in zip(o0[6], ref_rfr):
        assert np.allclose(cv_s, cv_r, atol=0.02) and abs(hold - hold_r) < 0.02, (cv_s, cv_r)


def test_shard_bounds_cover_rows():
    for n in (1, 7, 100, 1001):
        for w in (1, 2, 3, 8):
            b = [shard_bounds(n, w, r) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
            assert max(e - s for s, e in b) - min(e - s for s, e in b) <= 1


def _gpu_rank(rank, world, port, outq):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", OMP_NUM_THREADS="2")
    try:
        from cs230_distributed_machine_learning_amd.parallel import dist
        from cs230_distributed_machine_learning_amd.parallel.data_parallel import RowShard
        from cs230_distributed_machine_learning_amd.utils import native

        # both ranks share the one GPU of the test box; gloo carries the device tensors
        inf = dist.init(backend="gloo", want_gpu=True, timeout_s=120)
        native.hip_lib()
        X, y_cls, _ = _table(n=40000, d=48, seed=1)
        a, b = shard_bounds(len(X), world, rank)
        sh = RowShard(X[a:b], y_cls, a, True, inf.device)
        lr = _run(sh, X, y_cls, "LogisticRegression", GPU_GRID)
        knn = _run(sh, X, y_cls, "KNeighborsClassifier", KNN_GRID[:2], cv=3)
        # row-sharded boosting on the fused stage (phased gbrt.hip kernels + all-reduces)
        lib = native.hip_lib()
        phase_fn, calls = lib.dml_gb_stage_phase, []

        def counted(*a):
            calls.append(1)
            return phase_fn(*a)

        lib.dml_gb_stage_phase = counted
        Xg, yg_cls, yg_reg = _table(n=12000, d=10, seed=2)
        a, b = shard_bounds(len(Xg), world, rank)
        gbc = _run(RowShard(Xg[a:b], yg_cls, a, True, inf.device), Xg, yg_cls, "GradientBoostingClassifier",
                   GB_GPU_GRID, cv=3)
        gbr = _run(RowShard(Xg[a:b], yg_reg, a, False, inf.device), Xg, yg_reg, "GradientBoostingRegressor",
                   GBR_GPU_GRID, cv=3)
        outq.put(("ok", rank, lr, knn, gbc, gbr, len(calls)))
        dist.destroy()
    except Exception:  # pragma: no cover
        import traceback

        outq.put(("err", rank, traceback.format_exc()))


GB_GPU_GRID = [{"n_estimators": 10, "max_depth": 3, "learning_rate": 0.3, "random_state": 1},
               {"n_estimators": 6, "max_depth": 4, "subsample": 0.7, "random_state": 2}]
GBR_GPU_GRID = [{"n_estimators": 8, "max_depth": 3, "learning_rate": 0.3, "loss": loss, "random_state": 1}
                for loss in ("squared_error", "absolute_error", "huber", "quantile")] + \
               [{"n_estimators": 5, "max_depth": 9, "loss": "huber", "alpha": 0.7, "subsample": 0.8,
                 "random_state": 4}]
GPU_GRID = [{"C": c, "solver": "lbfgs", "max_iter": 60} for c in (0.01, 1.0)] + \
           [{"C": 0.3, "solver": "liblinear", "class_weight": "balanced", "max_iter": 60}]


@pytest.mark.gpu
def test_row_sharded_lr_on_gpu_matches_single_process():
    """MFMA objective on each rank's shard + gradient all-reduce == the one-GPU fit."""
    import torch

    from cs230_distributed_machine_learning_amd.data.device import DeviceData

    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gpu_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        outs = [q.get(timeout=300) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for o in outs:
        assert o[0] == "ok", o[2]
    X, y_cls, _ = _table(n=40000, d=48, seed=1)
    ref = _run(DeviceData(X, y_cls, True, torch.device("cuda:0")), X, y_cls, "LogisticRegression", GPU_GRID)
    o0, o1 = sorted(outs, key=lambda o: o[1])
    assert o0[2] == o1[2]
    for (cv_s, hold), (cv_r, hold_r) in zip(o0[2], ref):
        assert np.allclose(cv_s, cv_r, atol=2e-3), (cv_s, cv_r)
        assert abs(hold - hold_r) <= 2e-3
    # row-sharded KNN (torch distances per shard + exact merge) vs the one-GPU HIP search
    assert o0[3] == o1[3]
    ref_knn = _run(DeviceData(X, y_cls, True, torch.device("cuda:0")), X, y_cls, "KNeighborsClassifier",
                   KNN_GRID[:2], cv=3)
    for (cv_s, hold), (cv_r, hold_r) in zip(o0[3], ref_knn):
        assert np.allclose(cv_s, cv_r, atol=1e-3), (cv_s, cv_r)
    # row-sharded boosting: the fused stage ran on every rank; same scores on both ranks and
    # (regression trees from fp32 histograms summed over ranks: near-tie splits may differ)
    # close to the one-GPU fits
    assert o0[6] > 0 and o1[6] == o0[6]
    assert o0[4] == o1[4] and o0[5] == o1[5]
    Xg, yg_cls, yg_reg = _table(n=12000, d=10, seed=2)
    ref_gbc = _run(DeviceData(Xg, yg_cls, True, torch.device("cuda:0")), Xg, yg_cls, "GradientBoostingClassifier",
                   GB_GPU_GRID, cv=3)
    ref_gbr = _run(DeviceData(Xg, yg_reg, False, torch.device("cuda:0")), Xg, yg_reg, "GradientBoostingRegressor",
                   GBR_GPU_GRID, cv=3)
    for (cv_s, hold), (cv_r, hold_r) in zip(o0[4] + o0[5], ref_gbc + ref_gbr):
        assert np.allclose(cv_s, cv_r, atol=0.02) and abs(hold - hold_r) <= 0.02, (cv_s, cv_r)


def test_needs_whole_rows_routes_gbrt_losses_task_parallel():
    """GradientBoosting candidates the row-sharded booster rejects (leaf percentiles, the
    early-stopping validation split, monotonic bounds) are routed task-parallel by the cluster."""
    from cs230_distributed_machine_learning_amd.parallel.runner import needs_whole_rows

    for loss in ("absolute_error", "huber", "quantile"):
        assert needs_whole_rows("GradientBoostingRegressor", {"loss": loss})
    assert needs_whole_rows("GradientBoostingClassifier", {"n_iter_no_change": 5})
    assert needs_whole_rows("GradientBoostingRegressor", {"monotonic_cst": [1, 0]})
    assert not needs_whole_rows("GradientBoostingRegressor", {"loss": "squared_error"})
    # GPU workers: the fused stage's select all-reduces its byte counts (depth <= 10)
    assert not needs_whole_rows("GradientBoostingRegressor", {"loss": "huber", "max_depth": 5}, gpu=True)
    assert needs_whole_rows("GradientBoostingRegressor", {"loss": "quantile", "max_depth": 12}, gpu=True)
    assert needs_whole_rows("GradientBoostingRegressor", {"loss": "huber", "n_iter_no_change": 3}, gpu=True)
    assert not needs_whole_rows("GradientBoostingClassifier", {"loss": "log_loss", "n_iter_no_change": None})
    assert needs_whole_rows("RandomForestRegressor", {"criterion": "absolute_error"})
    assert not needs_whole_rows("LogisticRegression", {"C": 1.0})
