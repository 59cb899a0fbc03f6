"""HIP kernels of the non-forest families vs their plain-PyTorch fp32/fp64 references."""
import numpy as np
import pytest
import torch

from cs230_distributed_machine_learning_amd.data.device import DeviceData
from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates
from cs230_distributed_machine_learning_amd.search.cv import make_split_roles
from cs230_distributed_machine_learning_amd.search.grid import ParameterGrid

pytestmark = pytest.mark.gpu


def _dd(X, y, clf, dev, cv=5):
    dd = DeviceData(X, y, clf, dev)
    roles, names = make_split_roles(np.asarray(y), cv, clf, holdout=True, test_size=0.2, random_state=0)
    dd.set_splits(roles, names)
    return dd


@pytest.mark.parametrize("metric,p", [(0, 2.0), (1, 1.0), (2, float("inf")), (3, 3.0)])
@pytest.mark.parametrize("n,d,K", [(1000, 7, 5), (2053, 33, 64), (333, 3, 17)])
def test_knn_kernel_matches_torch(metric, p, n, d, K):
    from cs230_distributed_machine_learning_amd.models import neighbors as nb

    rng = np.random.RandomState(n + d)
    X = rng.randn(n, d).astype(np.float32)
    y = rng.randint(0, 3, n)
    dg = _dd(X, y, True, "cuda:0")
    splits = list(range(len(dg.split_names)))
    got = nb.knn_search_hip(dg, splits, K, metric, p)
    for s in splits:
        ref_d, ref_i = nb.knn_search_torch(dg.X.double(), dg.test_rows[s], dg.train_rows[s], K, metric, p)
        gd, gi = got[s]
        torch.testing.assert_close(gd.double(), ref_d, rtol=2e-5, atol=1e-5)
        # neighbour sets agree except where two distances are within float32 round-off
        mismatch = (gi != ref_i)
        if mismatch.any():
            close = (ref_d[mismatch] - gd.double()[mismatch]).abs() <= 1e-4 * ref_d[mismatch].abs().clamp_min(1)
            assert bool(close.all())


@pytest.mark.parametrize("n,d,K", [(1000, 7, 5), (5003, 33, 32), (2000, 150, 1), (3000, 20, 9)])
def test_knn_mfma_l2_equals_scalar_kernel(n, d, K, monkeypatch):
    """The matrix-core squared-L2 search (bf16x3 selection + exact re-rank) returns the
    scalar kernel's neighbours and distances bit for bit -- duplicate rows (exact ties)
    included."""
    from cs230_distributed_machine_learning_amd.models import neighbors as nb

    rng = np.random.RandomState(n + d)
    X = rng.randn(n, d).astype(np.float32) * rng.uniform(0.1, 10, d).astype(np.float32)
    X[n // 2:n // 2 + 50] = X[:50]                      # duplicates -> equal distances
    y = rng.randint(0, 3, n)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("DML_KNN_MFMA", mode)
        dg = _dd(X, y, True, "cuda:0")
        out[mode] = nb.knn_search_hip(dg, list(range(len(dg.split_names))), K, 0, 2.0)
    for s in out["0"]:
        assert torch.equal(out["1"][s][1], out["0"][s][1])
        assert torch.equal(out["1"][s][0], out["0"][s][0])


def test_knn_gpu_grid_matches_cpu():
    rng = np.random.RandomState(0)
    X = rng.randn(3000, 12).astype(np.float32)
    y = (X[:, 0] + 0.5 * X[:, 1] > 0).astype(int)
    grid = list(ParameterGrid({"n_neighbors": [1, 5, 31], "weights": ["uniform", "distance"]}))
    out = {}
    for dev in ("cpu", "cuda:0"):
        dd = DeviceData(X, y, True, dev)
        res = run_candidates(dd, JobSpec("KNeighborsClassifier", grid, cv=5), range(len(grid)))
        out[dev] = np.array([r.result["mean_cv_score"] for r in res])
    np.testing.assert_allclose(out["cuda:0"], out["cpu"], atol=1e-3)


@pytest.mark.parametrize("model,clf,loss", [("GradientBoostingClassifier", True, "log_loss"),
                                            ("GradientBoostingRegressor", False, "squared_error"),
                                            ("GradientBoostingRegressor", False, "huber")])
def test_gbrt_gpu_close_to_cpu(model, clf, loss):
    rng = np.random.RandomState(1)
    X = np.round(rng.randn(4000, 8), 1).astype(np.float32)
    if clf:
        y = (X[:, 0] * X[:, 1] + X[:, 2] > 0).astype(int)
    else:
        y = (X[:, 0] * 3 + X[:, 1] * X[:, 2] + rng.randn(4000) * 0.1).astype(np.float32)
    grid = list(ParameterGrid({"n_estimators": [10, 40], "max_depth": [2, 4], "loss": [loss]}))
    out = {}
    for dev in ("cpu", "cuda:0"):
        dd = DeviceData(X, y, clf, dev)
        res = run_candidates(dd, JobSpec(model, grid, cv=3), range(len(grid)))
        assert all(r.ok for r in res), [r.error for r in res]
        out[dev] = np.array([r.result["mean_cv_score"] for r in res])
    if loss == "squared_error":
        # exact integer regression histograms + a correctly rounded init: identical ensembles
        np.testing.assert_allclose(out["cuda:0"], out["cpu"], rtol=0, atol=1e-9)
    else:   # sigmoid / percentile / float64 index_add leaf updates differ in the last bits by device
        np.testing.assert_allclose(out["cuda:0"], out["cpu"], atol=5e-3)


@pytest.mark.parametrize("model,n_classes,loss,extra", [
    ("GradientBoostingClassifier", 3, "log_loss", {}),
    ("GradientBoostingClassifier", 2, "exponential", {}),
    ("GradientBoostingClassifier", 2, "log_loss", {}),
    ("GradientBoostingRegressor", 0, "squared_error", {}),
    ("GradientBoostingRegressor", 0, "absolute_error", {}),
    ("GradientBoostingRegressor", 0, "huber", {"alpha": [0.8]}),
    ("GradientBoostingRegressor", 0, "quantile", {"alpha": [0.3]}),
    ("GradientBoostingRegressor", 0, "absolute_error", {"subsample": [0.6]}),
    ("GradientBoostingRegressor", 0, "huber", {"subsample": [0.7]}),
    # deep trees: 1024 / 2048 path slots per tree
    ("GradientBoostingRegressor", 0, "squared_error", {"max_depth": [7, 10]}),
    ("GradientBoostingRegressor", 0, "quantile", {"max_depth": [9], "alpha": [0.4]}),
    ("GradientBoostingClassifier", 3, "log_loss", {"max_depth": [10]}),
    # early stopping on the percentile losses (huber's validation loss at the device delta)
    ("GradientBoostingRegressor", 0, "huber", {"n_iter_no_change": [2], "validation_fraction": [0.2]}),
    ("GradientBoostingRegressor", 0, "quantile", {"n_iter_no_change": [3], "alpha": [0.6]})])
def test_gbrt_fused_stage_matches_torch_stage(model, n_classes, loss, extra, monkeypatch, tmp_path):
    """The fused HIP stage (gbrt.hip: gradient, leaf line search -- Newton steps, or the exact
    radix-select leaf percentiles and huber delta -- raw update) against the torch stage on the
    same device: same CV scores, and -- with the models kept (the refit path) -- the same
    predictions from the stored artefacts."""
    from cs230_distributed_machine_learning_amd.engine.model_store import load_predictor, save_model

    rng = np.random.RandomState(3)
    X = np.round(rng.randn(3000, 6), 1).astype(np.float32)
    if n_classes:
        y = np.digitize(X[:, 0] + 0.5 * X[:, 1] * X[:, 2], [-0.5, 0.5][: n_classes - 1]).astype(int)
    else:
        y = (2 * X[:, 0] + X[:, 1] * X[:, 2] + 0.1 * rng.randn(3000)).astype(np.float32)
    grid = list(ParameterGrid({"n_estimators": [8, 20], "max_depth": [2, 4], "loss": [loss],
                               "learning_rate": [0.3], **extra}))
    out, preds = {}, {}
    from cs230_distributed_machine_learning_amd.utils import native

    lib = native.hip_lib()
    stage_fn, calls = lib.dml_gb_stage, []

    def counted(*args):
        calls.append(1)
        return stage_fn(*args)

    monkeypatch.setattr(lib, "dml_gb_stage", counted, raising=False)
    for flag in ("1", "0"):
        monkeypatch.setenv("DML_GB_FUSED", flag)
        n0 = len(calls)
        dd = _dd(X, y, bool(n_classes), "cuda:0", cv=3)
        spec = JobSpec(model, grid, cv=3, holdout=True, test_size=0.2, random_state=0, keep_models="all")
        res = run_candidates(dd, spec, range(len(grid)))
        assert all(r.ok for r in res), [r.error for r in res]
        assert (len(calls) > n0) == (flag == "1")   # the fused stage ran exactly when enabled
        out[flag] = np.array([r.result["mean_cv_score"] for r in res])
        preds[flag] = [load_predictor(save_model(r.model, str(tmp_path / f"m{flag}_{i}.npz"))).predict(X[:500])
                       for i, r in enumerate(res)]
    exact = loss in ("squared_error", "absolute_error", "quantile", "huber")
    np.testing.assert_allclose(out["1"], out["0"], rtol=0, atol=1e-9 if exact else 2e-3)
    for a, b in zip(preds["1"], preds["0"]):
        if n_classes:
            assert np.mean(a == b) >= 0.995
        else:
            np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("kg", [None, "24"])
@pytest.mark.parametrize("model,clf", [("GradientBoostingRegressor", False), ("GradientBoostingClassifier", True)])
def test_gbrt_root_count_cache_is_exact(model, clf, kg, monkeypatch):
    """Boosting builds reuse the roots' row-count histograms across stages (they only depend on
    the training rows): the ensembles are identical with and without the cache, one lane or two,
    with the large tier's packed count | w yq words, its compact 3-KB LDS slices or the 4-KB ones
    (DML_LARGE_NO_PACK, DML_LARGE_NO_COMPACT), and with row-window gathers for sparse nodes
    (DML_LARGE_FM_DIV)."""
    if kg is not None:   # feature groups wider than the pipelined loop's 16: the generic row loop
        monkeypatch.setenv("DML_TIER_KG_LARGE_REG", kg)
    rng = np.random.RandomState(4)
    X = rng.randn(200_000, 20).astype(np.float32)      # large-tier roots (> block_max rows)
    y = (X[:, 0] + X[:, 1] * X[:, 2] > 0).astype(int) if clf else (X[:, 0] + 0.3 * X[:, 3] ** 2).astype(np.float32)
    grid = list(ParameterGrid({"n_estimators": [6, 12], "max_depth": [3]}))
    out = {}
    for cache, lanes in (("0", "1"), ("1", "1"), ("1", "2"), ("1", "W"), ("0", "P"), ("0", "L")):
        monkeypatch.setenv("DML_GB_ROOT_CACHE", cache)
        monkeypatch.setenv("DML_GB_LANES", "1" if lanes in "LPW" else lanes)
        # row windows for nodes under n / 2 rows ("W"), or feature-major gathers everywhere
        monkeypatch.setenv("DML_LARGE_FM_DIV", "2" if lanes == "W" else "0")
        if lanes == "P":   # two atomics per (row, feature) instead of the packed count | w yq word
            monkeypatch.setenv("DML_LARGE_NO_PACK", "1")
        if lanes == "L":
            monkeypatch.setenv("DML_LARGE_NO_COMPACT", "1")
        dd = _dd(X, y, clf, "cuda:0", cv=3)
        res = run_candidates(dd, JobSpec(model, grid, cv=3), range(len(grid)))
        assert all(r.ok for r in res), [r.error for r in res]
        out[cache + lanes] = np.array([r.result["mean_cv_score"] for r in res])
    np.testing.assert_array_equal(out["11"], out["01"])
    np.testing.assert_array_equal(out["12"], out["01"])
    np.testing.assert_array_equal(out["1W"], out["01"])
    np.testing.assert_array_equal(out["0L"], out["01"])
    np.testing.assert_array_equal(out["0P"], out["01"])


def test_lr_link_grad_kernel_matches_torch():
    from cs230_distributed_machine_learning_amd.models import linear
    from cs230_distributed_machine_learning_amd.utils import native

    rng = np.random.RandomState(2)
    n, C = 5000, 4
    y = rng.randint(0, C, n).astype(np.int32)
    dd = _dd(rng.randn(n, 6).astype(np.float32), y, True, "cuda:0")
    S = len(dd.split_names)
    # fits: softmax (K=C), OvR (K=C), binary (K=1) on assorted splits
    kinds = [(linear.KIND_SOFTMAX, C), (linear.KIND_OVR, C), (linear.KIND_BINARY, 1)] * 3
    col0, K, kind, split, scale = [], [], [], [], []
    m = 0
    for i, (kd, k) in enumerate(kinds):
        col0.append(m); K.append(k); kind.append(kd); split.append(i % S); scale.append(1.0 / (i + 1))
        m += k
    Z = torch.randn(n, m, device="cuda:0")
    i32 = lambda v: torch.tensor(v, dtype=torch.int32, device="cuda:0")
    ycls = torch.from_numpy(y).cuda()
    R = torch.empty_like(Z)
    loss = torch.empty(len(kinds), dtype=torch.float64, device="cuda:0")
    lib = native.hip_lib()
    # keep every argument tensor alive across the asynchronous launch
    args = [i32(col0), i32(K), i32(kind), i32(split), torch.tensor(scale, dtype=torch.float32, device="cuda:0")]
    rc = lib.dml_lr_link_grad(native.ptr(Z), n, m, native.ptr(ycls), native.ptr(dd.roles),
                              *[native.ptr(a) for a in args], len(kinds), 0, 0, native.ptr(R), native.ptr(loss),
                              native.stream_handle())
    torch.cuda.synchronize()
    assert rc == 0
    Rr, lr = linear.link_grad_torch(Z.double(), ycls, dd.roles, col0, K, kind, split, scale)
    torch.testing.assert_close(R.double(), Rr, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(loss, lr, rtol=1e-4, atol=1e-4)


def _lr_batch(dd, specs):
    from cs230_distributed_machine_learning_amd.models import linear
    from cs230_distributed_machine_learning_amd.models.base import FitTask

    fam = linear.LogisticFamily()
    tasks = []
    for i, (params, split) in enumerate(specs):
        rp = fam.resolve("LogisticRegression", params, dd.n, dd.d, dd.n_classes)
        tasks.append(FitTask(task_id=i, candidate=i, split=split, model_type="LogisticRegression", params=rp))
    return fam, linear._Batch(dd, tasks)


@pytest.mark.parametrize("C_cls,n,d,fits,rt_gb", [(2, 3001, 70, 40, None), (3, 2500, 45, 40, None),
                                                  (4, 700, 300, 40, None), (2, 5003, 130, 300, None),
                                                  (3, 2100, 64, 130, None), (2, 5003, 130, 300, "0.004"),
                                                  (3, 2100, 64, 130, "0.002")])
def test_lr_mfma_objective_matches_fp32(C_cls, n, d, fits, rt_gb, monkeypatch):
    """Matrix-core (bf16x3) objective vs the fp32 GEMM + link-kernel path: loss and gradient.
    Batches of more than 256 columns run the 3-stage 256 x 128 kernels (k_lr_fwd3 / k_lr_grad3);
    ``rt_gb`` caps the residual buffer so the objective runs over several row chunks."""
    if rt_gb is not None:
        monkeypatch.setenv("DML_LR_RT_GB", rt_gb)
    from cs230_distributed_machine_learning_amd.models import linear

    rng = np.random.RandomState(C_cls * 7 + d)
    X = (rng.randn(n, d) * rng.uniform(0.1, 3.0, d)).astype(np.float32)
    y = rng.randint(0, C_cls, n)
    dd = _dd(X, y, True, "cuda:0")
    S = len(dd.split_names)
    specs = []
    for i in range(fits):   # softmax / OvR (liblinear) / class-weighted, assorted splits and C
        p = {"C": float(10.0 ** rng.uniform(-2, 2)), "solver": ["lbfgs", "liblinear"][i % 2]}
        if i % 5 == 0:
            p["class_weight"] = "balanced"
        specs.append((p, i % S))
    fam, b = _lr_batch(dd, specs)
    W = torch.randn((d + 1, b.M), device="cuda:0") * 0.05
    f0, G0 = fam._objective(dd, b, W)
    b.mf = linear.MfmaPlan(dd, b)
    assert b.mf.v3 == (b.M > 256)
    if rt_gb is not None:
        assert b.mf.n_chunks > 1
    f1, G1 = fam._objective(dd, b, W)
    torch.cuda.synchronize()
    torch.testing.assert_close(f1, f0, rtol=2e-5, atol=1e-6)
    scale = G0.abs().amax(0, keepdim=True).clamp_min(1e-6)
    assert float(((G1 - G0).abs() / scale).max()) < 2e-4


@pytest.mark.parametrize("rt_gb", [None, "0.004"])
def test_lr_mfma_skips_tiles_of_stopped_fits(rt_gb, monkeypatch):
    """With an ``active`` mask the v3 kernels skip column tiles whose fits all stopped; the
    loss and gradient of every active fit are bit-identical to the full evaluation."""
    if rt_gb is not None:
        monkeypatch.setenv("DML_LR_RT_GB", rt_gb)
    from cs230_distributed_machine_learning_amd.models import linear

    rng = np.random.RandomState(11)
    n, d = 5003, 130
    X = (rng.randn(n, d) * rng.uniform(0.1, 3.0, d)).astype(np.float32)
    y = rng.randint(0, 2, n)
    dd = _dd(X, y, True, "cuda:0")
    S = len(dd.split_names)
    Cs = 10.0 ** rng.uniform(-2, 2, 300)
    specs = [({"C": float(c), "solver": ["lbfgs", "liblinear"][i % 2]}, i % S) for i, c in enumerate(Cs)]
    fam, b = _lr_batch(dd, specs)
    b.mf = linear.MfmaPlan(dd, b)
    assert b.mf.v3
    W = torch.randn((d + 1, b.M), device="cuda:0") * 0.05
    f_all, G_all = fam._objective(dd, b, W)
    # stopped: every liblinear fit and the lbfgs fits of small C -> whole column tiles go idle
    act = torch.tensor([(i % 2 == 0) and c > 1.0 for i, c in enumerate(Cs)], device="cuda:0")
    f_act, G_act = fam._objective(dd, b, W, act)
    torch.cuda.synchronize()
    col_tiles = b.mf.Mp // linear._TILE
    assert 0 < int(b.mf.live[0]) < col_tiles
    assert torch.equal(f_act[act], f_all[act])
    cols = act[b.col_fit]
    assert torch.equal(G_act[:, cols], G_all[:, cols])
    f_again, G_again = fam._objective(dd, b, W)          # no mask: every tile again
    assert torch.equal(f_again, f_all) and torch.equal(G_again, G_all)
    # the solver's first evaluation (W = 0) skips the forward GEMM: same result
    W0 = torch.zeros_like(W)
    f0, G0 = fam._objective(dd, b, W0)
    f0z, G0z = fam._objective(dd, b, W0, w_zero=True)
    assert torch.equal(f0z, f0) and torch.equal(G0z, G0)
    # ... and the grouped fp32 start the solver actually uses agrees with it
    fg, Gg = fam._objective_at_zero(dd, b)
    torch.testing.assert_close(fg, f0, rtol=2e-5, atol=1e-6)
    assert float(((Gg - G0).abs() / G0.abs().amax(0, keepdim=True).clamp_min(1e-6)).max()) < 2e-4


def test_lr_mfma_fits_match_fp32_path(monkeypatch):
    """Whole batched L-BFGS solves on the matrix cores reach the fp32 path's CV scores."""
    rng = np.random.RandomState(5)
    X = rng.randn(30000, 40).astype(np.float32)
    y = (X @ rng.randn(40) + 2 * rng.randn(30000) > 0).astype(int)
    grid = list(ParameterGrid({"C": [0.001, 0.1, 10.0], "solver": ["lbfgs", "liblinear"]}))
    out = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("DML_LR_MFMA", flag)
        dd = DeviceData(X, y, True, "cuda:0")
        res = run_candidates(dd, JobSpec("LogisticRegression", grid, cv=5), range(len(grid)))
        assert all(r.ok for r in res), [r.error for r in res]
        out[flag] = np.array([r.result["mean_cv_score"] for r in res])
    np.testing.assert_allclose(out["1"], out["0"], atol=1e-3)


def test_lr_solve_skipping_stopped_fits_is_exact(monkeypatch):
    """A v3 batch (> 256 columns) solved with and without skipping stopped fits' tiles:
    identical fits (the skip only drops work whose results the solver never reads)."""
    rng = np.random.RandomState(8)
    X = rng.randn(20000, 40).astype(np.float32)
    y = (X @ rng.randn(40) + 2 * rng.randn(20000) > 0).astype(int)
    grid = [{"C": float(c), "solver": s} for c in 10.0 ** np.linspace(-3, 2, 30) for s in ("lbfgs", "liblinear")]
    out = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("DML_LR_SKIP_DONE", flag)
        dd = DeviceData(X, y, True, "cuda:0")
        res = run_candidates(dd, JobSpec("LogisticRegression", grid, cv=5), range(len(grid)))
        assert all(r.ok for r in res), [r.error for r in res]
        out[flag] = np.array([r.result["mean_cv_score"] for r in res])
    np.testing.assert_array_equal(out["1"], out["0"])


def test_lr_gpu_grid_matches_cpu():
    rng = np.random.RandomState(3)
    X = rng.randn(40000, 10).astype(np.float32)          # large enough for the device solver
    y = (X @ rng.randn(10) + rng.randn(40000) > 0).astype(int)
    grid = list(ParameterGrid({"C": [0.01, 1.0, 100.0], "solver": ["lbfgs", "liblinear"]}))
    out = {}
    for dev in ("cpu", "cuda:0"):
        dd = DeviceData(X, y, True, dev)
        res = run_candidates(dd, JobSpec("LogisticRegression", grid, cv=5), range(len(grid)))
        out[dev] = np.array([r.result["mean_cv_score"] for r in res])
    np.testing.assert_allclose(out["cuda:0"], out["cpu"], atol=2e-3)


@pytest.mark.parametrize("model,clf", [("SVC", True), ("SVR", False)])
def test_svm_gpu_matches_cpu_solver(model, clf):
    """The HIP SMO and the host SMO run the same algorithm: same dual solution."""
    from cs230_distributed_machine_learning_amd.models.base import FitTask, family_of

    rng = np.random.RandomState(5)
    n = 900
    X = rng.randn(n, 6).astype(np.float32)
    if clf:
        y = np.digitize(X[:, 0] + 0.5 * X[:, 1] ** 2 + 0.3 * rng.randn(n), [-0.5, 0.8])   # 3 classes
    else:
        y = (np.sin(X[:, 0]) + 0.3 * X[:, 1] + 0.1 * rng.randn(n)).astype(np.float32)
    grid = list(ParameterGrid({"C": [0.3, 3.0], "kernel": ["rbf", "poly", "linear"]}))
    out = {}
    for dev in ("cpu", "cuda:0"):
        dd = DeviceData(X, y, clf, dev)
        res = run_candidates(dd, JobSpec(model, grid, cv=3), range(len(grid)))
        assert all(r.ok for r in res), [r.error for r in res]
        out[dev] = np.array([r.result["mean_cv_score"] for r in res])
    np.testing.assert_allclose(out["cuda:0"], out["cpu"], atol=2e-3)


@pytest.mark.parametrize("model,slots", [("SVC", 4), ("SVC", 1024), ("SVR", 8)])
def test_svm_split_solver_equals_single_workgroup_solver(model, slots, monkeypatch):
    """Several workgroups per problem exchanging atomic records + the LRU column cache
    (evicting at 4 / 8 slots) take exactly the single-workgroup solver's SMO steps."""
    from cs230_distributed_machine_learning_amd.models.base import family_of

    rng = np.random.RandomState(7)
    n = 7000
    X = rng.randn(n, 9).astype(np.float32)
    clf = model == "SVC"
    y = (X[:, 0] + 0.4 * X[:, 1] ** 2 + 0.5 * rng.randn(n) > 0.3).astype(int) if clf else \
        (np.sin(X[:, 0]) + 0.2 * rng.randn(n)).astype(np.float32)
    grid = list(ParameterGrid({"C": [0.5, 5.0], "gamma": ["scale"]}))
    out, stats = {}, {}
    fam = family_of(model)
    for mode in ("0", "1"):
        monkeypatch.setenv("DML_SVM_SPLIT", mode)
        monkeypatch.setenv("DML_SVM_CACHE_SLOTS", str(slots))
        dd = DeviceData(X, y, clf, "cuda:0")
        res = run_candidates(dd, JobSpec(model, grid, cv=3, holdout=False), range(len(grid)))
        assert all(r.ok for r in res), [r.error for r in res]
        out[mode] = [r.result["cv_scores"] for r in res]
        stats[mode] = dict(fam.last_solve_stats)
    assert stats["1"]["solver"] == "split" and stats["1"]["workgroups_per_problem"] > 1, stats
    assert stats["1"]["iterations_max"] == stats["0"]["iterations_max"], stats
    assert out["1"] == out["0"]


def test_slice_metrics_report_gpu_fields():
    """J3 records of a device slice carry the GPU index, the slice's HBM working set and
    its fits/s (SURVEY §5.1/§5.5 observability fields)."""
    from cs230_distributed_machine_learning_amd.engine.service import run_slice

    rng = np.random.RandomState(5)
    X = rng.randn(4000, 12).astype(np.float32)
    y = (X[:, 0] + 0.3 * rng.randn(4000) > 0).astype(np.int64)
    dd = DeviceData(X, y, True, "cuda:0")
    plan = {"model_type": "RandomForestClassifier", "cv": 3, "scoring": None, "holdout": True, "test_size": 0.2,
            "random_state": 0, "error_score": float("nan")}
    params = [{"n_estimators": 8, "max_depth": 4}, {"n_estimators": 8, "max_depth": 8}]
    results, metrics, wall = run_slice(plan, params, ["s-0", "s-1"], dd, [0, 1], "rank0", "cuda:0")
    assert all(r.ok for r in results)
    for m in metrics.values():
        assert m["gpu_id"] == 0 and m["hbm_peak_bytes"] > 0
        assert m["slice_fits"] == 8 and m["slice_fits_per_s"] > 0


@pytest.mark.parametrize("n,d,offset", [(5000, 7, 0.0), (40000, 33, 500.0), (3000, 130, 3.0)])
def test_linreg_fused_moments_match_float64_torch(n, d, offset, monkeypatch):
    """LinearRegression's one-pass f64-MFMA split moments (dml_split_moments) give the
    float64 torch solution: same coefficients / predictions, with and without intercept,
    on data far from the origin (the shift keeps the centring exact)."""
    from cs230_distributed_machine_learning_amd.models import linear

    rng = np.random.RandomState(d)
    X = (rng.randn(n, d) + offset).astype(np.float32)
    y = (X @ rng.randn(d) + 0.1 * rng.randn(n) + 2.0).astype(np.float32)
    dg = _dd(X, y, False, "cuda:0")
    splits = list(range(len(dg.split_names)))
    M, shift = linear.LinearRegressionFamily.split_moments(dg, splits)
    Z = torch.cat([torch.from_numpy(X).double() - shift[:d].cpu(), torch.ones(n, 1, dtype=torch.float64),
                   torch.from_numpy(y).double().view(-1, 1) - shift[d].cpu()], 1)
    for i, s in enumerate(splits):
        m = torch.from_numpy((dg.roles[s] == 1).cpu().numpy()).double()
        ref = (Z * m[:, None]).t() @ Z
        torch.testing.assert_close(M[i].cpu(), ref, rtol=1e-10, atol=1e-7 * float(ref.abs().max()))
    fam = linear.LinearRegressionFamily()
    tasks = []
    from cs230_distributed_machine_learning_amd.models.base import FitTask
    for fi in (True, False):
        for s in splits:
            tasks.append(FitTask(task_id=len(tasks), candidate=0, split=s, model_type="LinearRegression",
                                 params=fam.resolve("LinearRegression", {"fit_intercept": fi}, n, d, 1)))
    got = fam.run(dg, tasks)
    monkeypatch.setenv("DML_LINREG_KERNEL", "0")
    ref = fam.run(dg, tasks)
    for a, b in zip(got, ref):
        torch.testing.assert_close(a.pred.double(), b.pred.double(), rtol=1e-5, atol=1e-4)


def test_pca_gpu_fused_covariance_matches_cpu():
    """PCA on the GPU takes every split's covariance from the fused moments kernel; the
    CV log-likelihood scores match the host float64 path."""
    rng = np.random.RandomState(3)
    X = (rng.randn(6000, 12) @ rng.randn(12, 12) + 40.0).astype(np.float32)
    y = rng.randint(0, 2, 6000)
    grid = list(ParameterGrid({"n_components": [1, 3, 6, 11], "whiten": [False, True]}))
    out = {}
    for dev in ("cpu", "cuda:0"):
        dd = DeviceData(X, y, True, dev)
        res = run_candidates(dd, JobSpec("PCA", grid, cv=5), range(len(grid)))
        assert all(r.ok for r in res), [r.error for r in res]
        out[dev] = np.array([r.result["mean_cv_score"] for r in res])
    np.testing.assert_allclose(out["cuda:0"], out["cpu"], rtol=1e-6, atol=1e-6)
