"""Row-sharded forest builder (ops/forest_dp.py, csrc/kernels/forest_dp.hip, forest_dp_cpu.cpp).

The level-synchronous builder takes every decision of the one-process builders
(forest_common.h), so on one rank it must grow node-for-node the trees of
``forest_ops.build_cpu``; shards over ranks are covered in tests/test_data_parallel.py
(gloo, CPU) and below on the GPU."""
import os
import socket

import numpy as np
import pytest
import torch

from cs230_distributed_machine_learning_amd.models.forest import native_seed
from cs230_distributed_machine_learning_amd.ops import binning, forest_dp, forest_ops
from cs230_distributed_machine_learning_amd.utils import native


def canon(fb, T):
    """Breadth-first (split, value) records of every tree: equal iff the trees are equal."""
    nodes = np.asarray(fb.nodes.cpu() if isinstance(fb.nodes, torch.Tensor) else fb.nodes)
    vals = np.asarray(fb.vals.cpu() if isinstance(fb.vals, torch.Tensor) else fb.vals)
    out = []
    for t in range(T):
        q, rec = [t], []
        while q:
            nq = []
            for i in q:
                rec.append((int(nodes[i, 0]), tuple(vals[i].tolist())))
                if nodes[i, 0] >= 0:
                    nq += [int(nodes[i, 1]), int(nodes[i, 1]) + 1]
            q = nq
        out.append(rec)
    return out


def _specs(T, d, crit=0, mf=None, md=2**31 - 1, msl=1, mss=2, boot=1, lam=1.0, mid=0.0, cw_mode=0, seed=0):
    s = forest_ops.make_specs(T)
    s["seed"] = [native_seed(seed, j) for j in range(T)]
    s["split"] = np.arange(T) % 2
    s["max_depth"], s["min_samples_split"], s["min_samples_leaf"] = md, mss, msl
    s["max_features"] = mf or max(1, int(np.sqrt(d)))
    s["bootstrap"], s["criterion"], s["min_impurity_decrease"] = boot, crit, mid
    s["pois_cdf"] = native.poisson_cdf_table(lam)
    s["cw_mode"] = cw_mode
    return s


def _data(n=2500, d=14, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, d)).astype(np.float32)
    X[:, 3] = rng.integers(0, 2, n)          # low-cardinality columns: constant in many nodes
    X[:, 5] = rng.integers(0, 3, n)
    X[:, 7] = 1.0                            # constant everywhere
    z = X[:, 0] + X[:, 3] + 0.5 * rng.normal(size=n)
    y = (z > 0.5).astype(np.int32) + (X[:, 1] > 1.0)
    yr = (2 * X[:, 0] + X[:, 5] + 0.1 * rng.normal(size=n)).astype(np.float32)
    E = binning.quantile_edges(torch.from_numpy(X))
    Xb = binning.bin_matrix(torch.from_numpy(X), E)
    roles = np.ones((2, n), np.uint8)
    roles[1, ::4] = 2
    _data.last = (X, E)
    return Xb, y, yr, roles


CASES = [
    dict(crit=0),
    dict(crit=1, md=7, msl=3),
    dict(crit=0, mf=14, mss=9, mid=1e-3),
    dict(crit=0, cw_mode=1, boot=0),
    dict(crit=1, cw_mode=2, lam=0.6),
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_dp_builder_one_rank_matches_cpu_builder(case):
    Xb, y, _, roles = _data()
    kw = CASES[case]
    T = 5
    specs = _specs(T, Xb.shape[1], **kw)
    cw = None
    if kw.get("cw_mode"):
        cw = np.tile(np.array([1.0, 2.5, 0.7]), (T, 1))
    ref = forest_ops.build_cpu(Xb.numpy(), y, None, roles, specs, 3, False, cw=cw)
    dp = forest_dp.build_dp(Xb, torch.from_numpy(y), None, torch.from_numpy(roles), specs, 3, False, 0,
                            cw=None if cw is None else cw.copy())
    assert canon(ref, T) == canon(dp, T)
    assert dp.stats["levels"] > 3


def test_dp_builder_search_rounds_and_chunks():
    """A tiny histogram budget splits every round into one-node all-reduce chunks, and
    max_features=1 with constant columns forces extra search rounds: same trees."""
    Xb, y, _, roles = _data(n=900)
    specs = _specs(3, Xb.shape[1], mf=1)
    ref = forest_ops.build_cpu(Xb.numpy(), y, None, roles, specs, 3, False)
    dp = forest_dp.build_dp(Xb, torch.from_numpy(y), None, torch.from_numpy(roles), specs, 3, False, 0,
                            hist_budget=1)
    assert canon(ref, 3) == canon(dp, 3)
    assert dp.stats["rounds"] > dp.stats["levels"]


def test_dp_builder_regression_one_rank():
    Xb, _, yr, roles = _data()
    specs = _specs(4, Xb.shape[1], crit=2, mf=14, msl=2)
    ref = forest_ops.build_cpu(Xb.numpy(), None, yr, roles, specs, 1, True)
    dp = forest_dp.build_dp(Xb, None, torch.from_numpy(yr), torch.from_numpy(roles), specs, 1, True, 0)
    n = Xb.shape[0]
    rows = np.arange(n, dtype=np.int32)
    pr = forest_ops.predict(ref, Xb.numpy(), np.array([0, 4]), np.array([0, n]), rows)
    pd = forest_ops.predict(dp.to_numpy(), Xb.numpy(), np.array([0, 4]), np.array([0, n]), rows)
    # exact integer regression sums (forest_common.h): the same trees, node for node
    assert canon(ref, 4) == canon(dp, 4)
    assert np.array_equal(pr, pd)


def test_dp_refine_matches_host_refine():
    """Midpoint thresholds on exactly-binned columns: global MIN of the right-going bins."""
    Xb, y, _, roles = _data()
    X = torch.from_numpy(np.round(np.random.default_rng(3).normal(size=Xb.shape) * 3).astype(np.float32))
    from cs230_distributed_machine_learning_amd.data.device import DeviceData

    dd = DeviceData(X, y, True)
    Xb = dd.binned()
    vals, exact = dd.bin_values()
    assert bool(exact.any())
    specs = _specs(3, Xb.shape[1])
    ref = forest_ops.build_cpu(Xb.numpy(), y, None, roles, specs, 3, False)
    forest_ops.refine_thresholds(ref, Xb.numpy(), specs, roles, vals.numpy(), exact.numpy())
    dp = forest_dp.build_dp(Xb, torch.from_numpy(y), None, torch.from_numpy(roles), specs, 3, False, 0)
    forest_dp.refine_dp(dp, Xb, torch.from_numpy(roles), specs, 0, vals, exact)
    assert canon(ref, 3) == canon(dp, 3)


# ---- GPU --------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("case", [0, 1, 4])
def test_dp_builder_gpu_matches_cpu_builder(case):
    """HIP histogram tiles (LDS) + small-node atomics + split/partition kernels == C++."""
    Xb, y, _, roles = _data(n=60000, d=40, seed=case)
    kw = dict(CASES[case])
    T = 6
    specs = _specs(T, Xb.shape[1], **kw)
    cw = np.tile(np.array([1.0, 2.5, 0.7]), (T, 1)) if kw.get("cw_mode") else None
    ref = forest_ops.build_cpu(Xb.numpy(), y, None, roles, specs, 3, False, cw=cw)
    dev = torch.device("cuda:0")
    X, E = _data.last
    Xg = binning.bin_matrix(torch.from_numpy(X).to(dev), E.to(dev))   # row-pitch padded device bins
    assert torch.equal(Xg.cpu(), Xb)
    dp = forest_dp.build_dp(Xg, torch.from_numpy(y).to(dev), None, torch.from_numpy(roles).to(dev), specs, 3, False,
                            0, cw=None if cw is None else cw.copy())
    assert dp.on_gpu
    assert canon(ref, T) == canon(dp, T)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gpu_rank(rank, world, port, outq):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", OMP_NUM_THREADS="2")
    try:
        from cs230_distributed_machine_learning_amd.parallel import dist
        from cs230_distributed_machine_learning_amd.parallel.data_parallel import RowShard, shard_bounds

        inf = dist.init(backend="gloo", want_gpu=True, timeout_s=120)
        X, y = _gpu_table()
        a, b = shard_bounds(len(X), world, rank)
        sh = RowShard(X[a:b], y, a, True, inf.device)
        outq.put(("ok", rank, _run_rf(sh), _run_rf(sh, "GradientBoostingClassifier", GB_GRID)))
        dist.destroy()
    except Exception:  # pragma: no cover
        import traceback

        outq.put(("err", rank, traceback.format_exc()))


def _gpu_table():
    rng = np.random.default_rng(11)
    X = rng.normal(size=(30000, 24)).astype(np.float32)
    y = (X[:, 0] - X[:, 2] + 0.6 * rng.normal(size=len(X)) > 0).astype(np.int64)
    return X, y


RF_GRID = [{"n_estimators": 6, "max_depth": md, "class_weight": cw, "random_state": 3}
           for md, cw in ((None, None), (9, "balanced"))]


GB_GRID = [{"n_estimators": 10, "max_depth": 3, "learning_rate": 0.3, "subsample": 0.8, "random_state": 4}]


def _run_rf(data, model="RandomForestClassifier", grid=RF_GRID):
    from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates

    spec = JobSpec(model, grid, cv=3, holdout=True, test_size=0.2, random_state=1, keep_models="none")
    res = run_candidates(data, spec, range(len(grid)))
    assert all(r.ok for r in res), [r.error for r in res if not r.ok]
    return [(r.result["cv_scores"], r.result.get("accuracy")) for r in res]


@pytest.mark.gpu
def test_row_sharded_forest_two_ranks_on_gpu():
    """Two ranks share the test box's GPU (gloo carries the device histograms): the
    row-sharded RF job scores exactly what the one-GPU task-parallel builder scores."""
    import torch.multiprocessing as mp

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
    X, y = _gpu_table()
    dd = DeviceData(X, y, True, torch.device("cuda:0"))
    ref = _run_rf(dd)
    o0, o1 = sorted(outs, key=lambda o: o[1])
    assert o0[2] == o1[2] == ref, (o0[2], ref)
    # row-sharded boosting (fp32 stage histograms summed across ranks): close to one GPU
    assert o0[3] == o1[3]
    for (cv_s, hold), (cv_r, hold_r) in zip(o0[3], _run_rf(dd, "GradientBoostingClassifier", GB_GRID)):
        assert np.allclose(cv_s, cv_r, atol=0.02) and abs(hold - hold_r) <= 0.02, (cv_s, cv_r)


def _w3_data():
    rng = np.random.default_rng(5)
    X = rng.normal(size=(7001, 9)).astype(np.float32)
    X[:, 2] = rng.integers(0, 3, 7001)
    y = ((X[:, 0] + X[:, 2] + rng.normal(size=7001)) > 0.7).astype(np.int64) + (X[:, 1] > 1)
    return X, y


def _w3_yreg(X):
    return (X[:, 0] * 3 + X[:, 1] * X[:, 3] + 0.25 * X[:, 2]).astype(np.float32)


def _w3_rank(rank, world, port, outq):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), OMP_NUM_THREADS="2")
    try:
        from cs230_distributed_machine_learning_amd.parallel import dist
        from cs230_distributed_machine_learning_amd.parallel.data_parallel import RowShard, shard_bounds

        inf = dist.init(want_gpu=False, timeout_s=120)
        X, y = _w3_data()
        a, b = shard_bounds(len(X), world, rank)
        sh = RowShard(X[a:b], y, a, True, inf.device)
        sh.set_splits(np.ones((1, len(X)), np.uint8), ["full"])
        specs = _specs(5, 9, crit=1, mf=3)
        specs["split"] = 0
        fb = forest_dp.build_dp(sh.binned(), sh.y_cls, None, sh.roles, specs, 3, False, sh.r0, reduce=sh.all_reduce,
                                comm=sh)
        # regression: integer histogram / root sums summed over the ranks (exact)
        shr = RowShard(X[a:b], _w3_yreg(X), a, False, inf.device)
        shr.set_splits(np.ones((1, len(X)), np.uint8), ["full"])
        rspecs = _specs(4, 9, crit=2, mf=4, msl=2)
        rspecs["split"] = 0
        fr = forest_dp.build_dp(shr.binned(), None, shr.y_reg, shr.roles, rspecs, 1, True, shr.r0,
                                reduce=shr.all_reduce, comm=shr)
        outq.put(("ok", rank, canon(fb, 5), canon(fr, 4)))
        dist.destroy()
    except Exception:  # pragma: no cover
        import traceback

        outq.put(("err", rank, traceback.format_exc()))


def test_dp_builder_three_ranks_gloo():
    """Odd world size: node ownership padded to a multiple of 3, sparse small-node gathers
    of unequal length -- every rank grows the one-process trees."""
    import torch.multiprocessing as mp

    from cs230_distributed_machine_learning_amd.data.device import DeviceData

    X, y = _w3_data()
    dd = DeviceData(X, y, True)
    specs = _specs(5, 9, crit=1, mf=3)
    specs["split"] = 0
    ref = canon(forest_ops.build_cpu(dd.binned().numpy(), dd.y_enc, None, np.ones((1, len(X)), np.uint8), specs, 3,
                                     False), 5)
    rspecs = _specs(4, 9, crit=2, mf=4, msl=2)
    rspecs["split"] = 0
    rref = canon(forest_ops.build_cpu(dd.binned().numpy(), None, _w3_yreg(X), np.ones((1, len(X)), np.uint8), rspecs,
                                      1, True), 4)
    world, port = 3, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_w3_rank, args=(r, world, port, q)) for r in range(world)]
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
        assert o[2] == ref
        assert o[3] == rref   # row-sharded regression trees == the one-process trees


def test_dp_builder_tree_chunks_concatenate_to_one_pool():
    """tree_chunk: trees grown a few at a time land in the one-build pool layout."""
    Xb, y, _, roles = _data(n=1500)
    T = 7
    specs = _specs(T, Xb.shape[1], cw_mode=2)
    cw = np.ones((T, 3))
    ref = forest_ops.build_cpu(Xb.numpy(), y, None, roles, specs, 3, False, cw=cw.copy())
    dp = forest_dp.build_dp(Xb, torch.from_numpy(y), None, torch.from_numpy(roles), specs, 3, False, 0,
                            cw=cw.copy(), tree_chunk=3)
    assert dp.stats["tree_chunks"] == 3
    assert canon(ref, T) == canon(dp, T)
    n = Xb.shape[0]
    rows = np.arange(n, dtype=np.int32)
    toff, roff = np.array([0, 3, T]), np.array([0, n // 2, n])
    assert np.array_equal(forest_ops.predict(ref, Xb.numpy(), toff, roff, rows),
                          forest_ops.predict(dp.to_numpy(), Xb.numpy(), toff, roff, rows))


@pytest.mark.gpu
def test_dp_builder_gpu_regression_and_poisson():
    """Regression (integer LDS tiles + 64-bit atomics, sequential-bin split kernel) and
    Poisson on the GPU vs the C++ builder: exact integer sums, identical trees."""
    Xb, _, yr, roles = _data(n=50000, d=20, seed=3)
    X, E = _data.last
    dev = torch.device("cuda:0")
    Xg = binning.bin_matrix(torch.from_numpy(X).to(dev), E.to(dev))
    n = Xb.shape[0]
    rows = np.arange(n, dtype=np.int32)
    for crit, y in ((2, yr), (3, np.exp(yr / np.abs(yr).max()).astype(np.float32))):
        specs = _specs(4, 20, crit=crit, mf=10, msl=3)
        ref = forest_ops.build_cpu(Xb.numpy(), None, y, roles, specs, 1, True)
        dp = forest_dp.build_dp(Xg, None, torch.from_numpy(y).to(dev), torch.from_numpy(roles).to(dev), specs, 1,
                                True, 0)
        pr = forest_ops.predict(ref, Xb.numpy(), np.array([0, 4]), np.array([0, n]), rows)
        pd = forest_ops.predict(dp, Xg, np.array([0, 4]), np.array([0, n]), torch.from_numpy(rows).to(dev)).cpu().numpy()
        assert canon(ref, 4) == canon(dp, 4), crit
        assert np.array_equal(pd, pr), crit
