"""HIP forest builder vs the C++ CPU builder (exact tree equality) and vs sklearn."""
import numpy as np
import pytest
import torch

from cs230_distributed_machine_learning_amd.ops import binning, forest_ops
from cs230_distributed_machine_learning_amd.search.cv import make_split_roles
from cs230_distributed_machine_learning_amd.utils import native

pytestmark = pytest.mark.gpu


def _specs(n_fits, ntrees, d, **kw):
    specs = forest_ops.make_specs(n_fits * ntrees)
    for f in range(n_fits):
        for t in range(ntrees):
            s = specs[f * ntrees + t]
            s["seed"] = 1000 + t
            s["split"] = f
            s["fit"] = f
            s["max_depth"] = kw.get("max_depth", 2**31 - 1)
            s["min_samples_split"] = kw.get("mss", 2)
            s["min_samples_leaf"] = kw.get("msl", 1)
            s["max_features"] = kw.get("k", max(1, int(np.sqrt(d))))
            s["bootstrap"] = kw.get("bootstrap", 1)
            s["criterion"] = kw.get("criterion", 0)
            s["min_impurity_decrease"] = kw.get("mid", 0.0)
            s["min_weight_frac"] = kw.get("mwf", 0.0)
            s["pois_cdf"] = native.poisson_cdf_table(1.0)
    return specs


def _canon(nodes, vals, T):
    """Canonical pre-order encoding of each tree (independent of node numbering)."""
    out = []
    for t in range(T):
        seq = []
        stack = [t]
        while stack:
            i = stack.pop()
            s, l = int(nodes[i, 0]), int(nodes[i, 1])
            seq.append((s, tuple(np.round(vals[i], 6))))
            if s >= 0:
                stack.append(l + 1)
                stack.append(l)
        out.append(seq)
    return out


def _data(n, d, n_classes=2, seed=0):
    from sklearn.datasets import make_classification

    X, y = make_classification(n_samples=n, n_features=d, n_informative=max(2, d // 2), n_classes=n_classes,
                               random_state=seed)
    return X.astype(np.float32), y


TIERS = [
    dict(sub_max=64, wave_max=256, block_max=2048, chunk=1024),
    dict(sub_max=32, wave_max=200, block_max=1024, chunk=512),
    dict(sub_max=0, wave_max=64, block_max=4096, chunk=2048),
    # the big-subtree tier (k_bigsub, binary builds; off by default)
    dict(sub_max=64, wave_max=256, block_max=2048, chunk=1024, bigsub_max=256),
    dict(sub_max=32, wave_max=200, block_max=1024, chunk=512, bigsub_max=200),
]


@pytest.mark.parametrize("words", ["packed", "plain"])
@pytest.mark.parametrize("tiers", range(len(TIERS)))
@pytest.mark.parametrize("n,d,C,kw", [
    (3000, 12, 2, {}),
    (20000, 20, 3, {"msl": 3}),
    (60000, 16, 2, {"max_depth": 12, "k": 16, "bootstrap": 0}),
    (5000, 30, 4, {"criterion": 0, "mss": 10}),
    (8000, 14, 3, {"criterion": 1}),            # entropy: host/device-identical log2 (forest_common.h)
    (20000, 16, 2, {"mwf": 0.002}),              # min_weight_fraction_leaf in every tier
    (6000, 12, 3, {"mwf": 0.02, "criterion": 1}),
])
def test_gpu_trees_match_cpu(n, d, C, kw, tiers, words, monkeypatch):
    if words == "plain":   # row ids only (the path for tables too tall for packed row words)
        monkeypatch.setenv("DML_ROW_WORDS_OFF", "1")
    X, y = _data(n, d, C)
    dev = torch.device("cuda:0")
    Xt = torch.from_numpy(X).to(dev)
    edges = binning.quantile_edges(Xt)
    Xb = binning.bin_matrix(Xt, edges)
    Xb_cpu = binning.bin_matrix(torch.from_numpy(X), edges.cpu()).numpy()
    assert np.array_equal(Xb.cpu().numpy(), Xb_cpu)
    roles, _ = make_split_roles(y, 3, True, holdout=False)
    specs = _specs(3, 6, d, **kw)
    ycls = y.astype(np.int32)
    g = forest_ops.build_gpu(Xb, torch.from_numpy(ycls).to(dev), None, torch.from_numpy(roles).to(dev), specs, C, False,
                             forest_ops.ForestTiers(**TIERS[tiers]))
    c = forest_ops.build_cpu(Xb_cpu, ycls, None, roles, specs, C, False)
    # the GPU pool may hold unreferenced slots (subtree kernels reserve node pairs in bulk):
    # compare the reachable trees
    gc = _canon(g.nodes.cpu().numpy(), g.vals.cpu().numpy(), len(specs))
    cc = _canon(c.nodes, c.vals, len(specs))
    assert sum(map(len, gc)) == sum(map(len, cc)) == c.stats["nodes"]
    assert gc == cc
    # predictions identical
    rows, roff = [], [0]
    for f in range(3):
        r = np.nonzero(roles[f] == 2)[0]
        rows.append(r)
        roff.append(roff[-1] + len(r))
    rows = np.concatenate(rows).astype(np.int32)
    roff = np.array(roff)
    toff = np.arange(4) * 6
    pg = forest_ops.predict(g, Xb, toff, roff, torch.from_numpy(rows).to(dev)).cpu().numpy()
    pc = forest_ops.predict(c, Xb_cpu, toff, roff, rows)
    assert np.array_equal(pg, pc)
    sg = forest_ops.score_stats(torch.from_numpy(rows).to(dev), roff, torch.from_numpy(pg).to(dev),
                                ycls=torch.from_numpy(ycls).to(dev))
    sc = forest_ops.score_stats(rows, roff, pc, ycls=ycls)
    assert np.allclose(sg, sc)


def test_gpu_big_block_tier_matches_cpu():
    """block_max above 32768: block-tier nodes with more than 2 x 256 row groups take the
    streaming partition (the two-pass one ranks at most 2 groups per thread)."""
    n, d, C = 150_000, 12, 2
    X, y = _data(n, d, C)
    dev = torch.device("cuda:0")
    edges = binning.quantile_edges(torch.from_numpy(X))
    Xb_cpu = binning.bin_matrix(torch.from_numpy(X), edges).numpy()
    Xb = torch.from_numpy(Xb_cpu).to(dev)
    roles, _ = make_split_roles(y, 3, True, holdout=False)
    specs = _specs(3, 2, d, max_depth=6)
    ycls = y.astype(np.int32)
    g = forest_ops.build_gpu(Xb, torch.from_numpy(ycls).to(dev), None, torch.from_numpy(roles).to(dev), specs, C, False,
                             forest_ops.ForestTiers(block_max=1 << 17))
    assert g.stats["tier_nodes"][2] > 0 and g.stats["tier_nodes"][3] == 0
    c = forest_ops.build_cpu(Xb_cpu, ycls, None, roles, specs, C, False)
    assert _canon(g.nodes.cpu().numpy(), g.vals.cpu().numpy(), len(specs)) == _canon(c.nodes, c.vals, len(specs))


@pytest.mark.parametrize("tiers", range(len(TIERS)))
@pytest.mark.parametrize("n,d,C", [(4000, 12, 2), (30000, 16, 3)])
def test_gpu_class_weighted_trees_match_cpu(n, d, C, tiers):
    """class_weight: dict weights (cw_mode 1) and balanced_subsample (cw_mode 2, weights
    computed by the root kernel from each tree's bootstrap counts) give identical trees."""
    X, y = _data(n, d, C, seed=3)
    y = np.where(np.random.RandomState(0).rand(n) < 0.6, 0, y)       # imbalanced
    dev = torch.device("cuda:0")
    edges = binning.quantile_edges(torch.from_numpy(X).to(dev))
    Xb = binning.bin_matrix(torch.from_numpy(X).to(dev), edges)
    Xb_cpu = Xb.cpu().numpy()
    roles, _ = make_split_roles(y, 3, True, holdout=False)
    specs = _specs(3, 6, d, msl=2)
    T = len(specs)
    cw = np.ones((T, C))
    for t in range(T):
        specs[t]["cw_mode"] = (0, 1, 2)[t % 3]
        if t % 3 == 1:
            cw[t] = 1.0 + np.arange(C) * 2.5
    ycls = y.astype(np.int32)
    g = forest_ops.build_gpu(Xb, torch.from_numpy(ycls).to(dev), None, torch.from_numpy(roles).to(dev), specs, C, False,
                             forest_ops.ForestTiers(**TIERS[tiers]), cw=cw.copy())
    c = forest_ops.build_cpu(Xb_cpu, ycls, None, roles, specs, C, False, cw=cw.copy())
    gc = _canon(g.nodes.cpu().numpy(), g.vals.cpu().numpy(), T)
    cc = _canon(c.nodes, c.vals, T)
    assert gc == cc


@pytest.mark.parametrize("is_reg", [False, True])
def test_gpu_max_leaf_prune_matches_cpu(is_reg):
    """max_leaf_nodes: the HIP best-first pass (one lane per tree) keeps the same nodes as
    the C++ one, and every limited tree ends with at most L leaves."""
    n, d, C = 20000, 16, 3
    X, y = _data(n, d, C, seed=4)
    dev = torch.device("cuda:0")
    Xb = binning.bin_matrix(torch.from_numpy(X).to(dev), binning.quantile_edges(torch.from_numpy(X).to(dev)))
    Xb_cpu = Xb.cpu().numpy()
    roles, _ = make_split_roles(y, 3, True, holdout=False)
    specs = _specs(3, 8, d, criterion=2 if is_reg else 1)
    T = len(specs)
    limit = np.array([(0, 2, 7, 40, 3000)[t % 5] for t in range(T)], dtype=np.int32)
    if is_reg:
        yr = (X[:, 0] * 2 + X[:, 1] ** 2).astype(np.float32)
        g = forest_ops.build_gpu(Xb, None, torch.from_numpy(yr).to(dev), torch.from_numpy(roles).to(dev), specs, 1, True)
        c = forest_ops.build_cpu(Xb_cpu, None, yr, roles, specs, 1, True)
    else:
        ycls = y.astype(np.int32)
        g = forest_ops.build_gpu(Xb, torch.from_numpy(ycls).to(dev), None, torch.from_numpy(roles).to(dev), specs, C,
                                 False)
        c = forest_ops.build_cpu(Xb_cpu, ycls, None, roles, specs, C, False)
    lg = forest_ops.prune_max_leaves(g, specs, limit)
    lc = forest_ops.prune_max_leaves(c, specs, limit)
    for lv in (lg, lc):
        assert all(lv[t] == -1 if limit[t] == 0 else 1 <= lv[t] <= limit[t] for t in range(T))
    gn = g.nodes.cpu().numpy()
    for t in range(T):   # the reported leaf count is the reachable one
        if limit[t]:
            assert sum(1 for s, _ in _canon(gn, g.vals.cpu().numpy(), t + 1)[t] if s < 0) == lg[t]
    assert np.array_equal(lg, lc)   # regression sums are exact integers too (forest_common.h)
    assert _canon(gn, g.vals.cpu().numpy(), T) == _canon(c.nodes, c.vals, T)


@pytest.mark.parametrize("words,crit,mid", [("packed", 2, 0.0), ("plain", 2, 0.0), ("packed", 3, 0.0),
                                            ("packed", 5, 200.0), ("packed", 2, 200.0), ("plain", 5, 50.0)])
def test_gpu_regression_trees_match_cpu(words, crit, mid, monkeypatch):
    """Regression histograms are exact 64-bit integer sums (forest_common.h fixed point) in
    every HIP tier, so GPU regression trees equal the C++ builder's node for node --
    squared_error, Poisson (crit 3) and friedman_mse (crit 5) -- with and without
    min_impurity_decrease (accept_improvement), and two builds are identical."""
    from sklearn.datasets import make_regression

    if words == "plain":
        monkeypatch.setenv("DML_ROW_WORDS_OFF", "1")
    X, y = make_regression(n_samples=8000, n_features=10, noise=5.0, random_state=1)
    X = X.astype(np.float32)
    y = (y + 300.0).astype(np.float32)   # mean far from zero: the old Sum wy^2 / w - mean^2 cancellation
    if crit == 3:
        y = np.exp((y - 300.0) / np.abs(y - 300.0).max() * 2).astype(np.float32)
    dev = torch.device("cuda:0")
    Xt = torch.from_numpy(X).to(dev)
    edges = binning.quantile_edges(Xt)
    Xb = binning.bin_matrix(Xt, edges)
    roles, _ = make_split_roles(y, 3, False, holdout=False)
    specs = _specs(3, 8, 10, k=10, criterion=crit)
    specs["min_impurity_decrease"] = mid
    T = len(specs)
    tiers = forest_ops.ForestTiers(**TIERS[0])   # small tiers: every tier (large included) grows nodes
    g = forest_ops.build_gpu(Xb, None, torch.from_numpy(y).to(dev), torch.from_numpy(roles).to(dev), specs, 1, True,
                             tiers)
    g2 = forest_ops.build_gpu(Xb, None, torch.from_numpy(y).to(dev), torch.from_numpy(roles).to(dev), specs, 1, True,
                              tiers)
    c = forest_ops.build_cpu(Xb.cpu().numpy(), None, y, roles, specs, 1, True)
    gc = _canon(g.nodes.cpu().numpy(), g.vals.cpu().numpy(), T)
    assert gc == _canon(c.nodes, c.vals, T)
    assert gc == _canon(g2.nodes.cpu().numpy(), g2.vals.cpu().numpy(), T)   # deterministic
    if mid > 0:   # the decrease test cut the trees (reachable nodes; the GPU pool reserves slots)
        full = forest_ops.build_cpu(Xb.cpu().numpy(), None, y, roles, _specs(3, 8, 10, k=10, criterion=crit), 1, True)
        assert sum(map(len, gc)) < 0.9 * sum(map(len, _canon(full.nodes, full.vals, T)))
    rows, roff = [], [0]
    for f in range(3):
        r = np.nonzero(roles[f] == 2)[0]
        rows.append(r)
        roff.append(roff[-1] + len(r))
    rows = np.concatenate(rows).astype(np.int32)
    roff = np.array(roff)
    toff = np.arange(4) * 8
    pg = forest_ops.predict(g, Xb, toff, roff, torch.from_numpy(rows).to(dev)).cpu().numpy()
    pc = forest_ops.predict(c, Xb.cpu().numpy(), toff, roff, rows)
    assert np.array_equal(pg, pc)


def test_wave_primitives_sort_and_scan():
    """DPP / permlane / readlane wave primitives (wave_ops.h) against numpy."""
    import ctypes

    lib = native.hip_lib()
    fn = lib.dml_test_wave_prims
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    rng = np.random.RandomState(0)
    x = rng.randint(0, 1 << 14, size=(16, 64)).astype(np.uint32)
    x[3] = 7  # all equal
    x[4] = np.arange(64)[::-1]
    xd = torch.from_numpy(x.astype(np.int32)).cuda()
    out = torch.empty((16, 11, 64), dtype=torch.int32, device="cuda")
    assert fn(xd.data_ptr(), out.data_ptr(), 16, native.stream_handle()) == 0
    torch.cuda.synchronize()
    o = out.cpu().numpy().view(np.uint32)
    lanes = np.arange(64)
    for bi in range(16):
        v = x[bi]
        assert np.array_equal(o[bi, 0], np.sort(v))
        assert np.array_equal(o[bi, 1], np.cumsum(v.astype(np.uint64)).astype(np.uint32))
        for k, m in enumerate((1, 2, 4, 8, 16, 32)):
            assert np.array_equal(o[bi, 2 + k], v[lanes ^ m]), (bi, m)
        g = v % 97
        assert (o[bi, 8] == np.flatnonzero(g == g.max())[0]).all()
        sd = np.concatenate([v[1:], [np.uint32(0xFFFFFFFF)]])
        assert np.array_equal(o[bi, 9], sd)
        mn = min((int(v[l]) << 32) | l for l in range(64))
        assert (o[bi, 10] == np.uint32(mn & 0xFFFFFFFF)).all()


@pytest.mark.gpu
def test_gpu_family_scores_match_host_path():
    """The whole forest family path on the GPU (build, refine, batched predict, fused
    scoring) gives the C++ host builder + predictor's CV and holdout scores, and exported
    models keep plain leaf records."""
    from cs230_distributed_machine_learning_amd.data.device import DeviceData
    from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates

    rng = np.random.RandomState(11)
    X = rng.randn(6000, 12).astype(np.float32)
    y = (X[:, 0] - X[:, 3] * X[:, 4] + 0.7 * rng.randn(6000) > 0).astype(np.int64)
    cands = [{"n_estimators": 9, "max_depth": md, "min_samples_leaf": msl} for md in (4, None) for msl in (1, 5)]
    spec = JobSpec("RandomForestClassifier", cands, cv=3, holdout=True, test_size=0.25, random_state=1,
                   keep_models="all")
    gpu = run_candidates(DeviceData(X, y, True, "cuda:0"), spec, range(len(cands)))
    cpu = run_candidates(DeviceData(X, y, True, "cpu"), spec, range(len(cands)))
    for g, c in zip(gpu, cpu):
        assert g.ok and c.ok
        # identical predictions; the two scoring paths may round the mean in the last ulp
        assert np.allclose(g.result["cv_scores"], c.result["cv_scores"], rtol=0, atol=1e-12)
        assert abs(g.result["accuracy"] - c.result["accuracy"]) <= 1e-12
        nodes = np.asarray(g.model["nodes"])
        assert set(np.unique(nodes[nodes[:, 0] < 0, 0]).tolist()) == {-1}


@pytest.mark.gpu
def test_gpu_predict_proba_matches_cpu():
    """predict_proba (probability scorers): the HIP predict kernel's class fractions equal
    the C++ predictor's for the same trees."""
    X, y = _data(20000, 12, 3)
    dev = torch.device("cuda:0")
    Xt = torch.from_numpy(X).to(dev)
    edges = binning.quantile_edges(Xt)
    Xb = binning.bin_matrix(Xt, edges)
    Xb_cpu = binning.bin_matrix(torch.from_numpy(X), edges.cpu()).numpy()
    roles, _ = make_split_roles(y, 3, True, holdout=False)
    specs = _specs(3, 6, 12, msl=4)
    ycls = y.astype(np.int32)
    c = forest_ops.build_cpu(Xb_cpu, ycls, None, roles, specs, 3, False)
    g = forest_ops.ForestBuild(torch.from_numpy(c.nodes).to(dev), torch.from_numpy(c.vals).to(dev), c.n_trees, c.VC,
                               False, 3)
    rows, roff = [], [0]
    for f in range(3):
        r = np.nonzero(roles[f] == 2)[0]
        rows.append(r)
        roff.append(roff[-1] + len(r))
    rows = np.concatenate(rows).astype(np.int32)
    roff, toff = np.array(roff), np.arange(4) * 6
    pg, qg = forest_ops.predict(g, Xb, toff, roff, torch.from_numpy(rows).to(dev), want_proba=True)
    pc, qc = forest_ops.predict(c, Xb_cpu, toff, roff, rows, want_proba=True)
    assert np.array_equal(pg.cpu().numpy(), pc)
    assert np.allclose(qg.cpu().numpy(), qc, atol=1e-6)
    assert np.allclose(qc.sum(1), 1.0, atol=1e-5)


@pytest.mark.gpu
def test_gpu_absolute_error_family_matches_host_path():
    """criterion='absolute_error' on device-resident data: the GPU MAE builder grows the
    trees (forest_mae.hip), then pruning, refine and the HIP predict + scoring run on the
    GPU -- the same CV scores as the all-host path, and a mixed MAE / squared_error grid
    keeps each candidate's own criterion."""
    from cs230_distributed_machine_learning_amd.data.device import DeviceData
    from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates

    rng = np.random.RandomState(5)
    X = rng.randint(0, 16, size=(3000, 6)).astype(np.float32)
    y = X[:, 0] - 0.5 * X[:, 2] + rng.standard_t(2, 3000)
    cands = [{"n_estimators": 4, "criterion": c, "max_depth": 6, "ccp_alpha": a}
             for c in ("absolute_error", "squared_error") for a in (0.0, 0.01)]
    spec = JobSpec("RandomForestRegressor", cands, cv=3, holdout=False, random_state=1)
    gpu = run_candidates(DeviceData(X, y, False, "cuda:0"), spec, range(len(cands)))
    cpu = run_candidates(DeviceData(X, y, False, "cpu"), spec, range(len(cands)))
    for i, (g, c) in enumerate(zip(gpu, cpu)):
        assert g.ok and c.ok
        # absolute_error: trees equal to the host builder's, predicted by the HIP kernel; the
        # squared_error candidates come from the GPU builder, whose float histogram sums
        # make trees close to, not equal to, the host's (test_gpu_regression_close_to_cpu)
        tol = 1e-6 if cands[i]["criterion"] == "absolute_error" else 2e-2
        assert np.allclose(g.result["cv_scores"], c.result["cv_scores"], rtol=0, atol=tol), (i, g.result, c.result)
    assert not np.allclose(cpu[0].result["cv_scores"], cpu[2].result["cv_scores"])


@pytest.mark.gpu
@pytest.mark.parametrize("tiers", range(len(TIERS)))
@pytest.mark.parametrize("is_reg", [False, True])
def test_gpu_monotonic_cst_trees_match_cpu(is_reg, tiers):
    """monotonic_cst on the HIP builder: the constrained-split rejection, the children's
    middle-value bounds and the final clip in every tier (subtree / wave / block / large)
    give the host builder's trees node for node (regression and binary classification)."""
    rng = np.random.RandomState(7)
    n, d = 12000, 8
    X = rng.randn(n, d).astype(np.float32)
    if is_reg:
        y = (2 * X[:, 0] - X[:, 1] + np.sin(3 * X[:, 2]) + 0.5 * rng.randn(n)).astype(np.float32)
    else:
        y = (X[:, 0] - 0.7 * X[:, 1] + rng.randn(n) > 0).astype(np.int32)
    dev = torch.device("cuda:0")
    Xb = binning.bin_matrix(torch.from_numpy(X).to(dev), binning.quantile_edges(torch.from_numpy(X).to(dev)))
    Xb_cpu = Xb.cpu().numpy()
    roles, _ = make_split_roles(y, 3, not is_reg, holdout=False)
    specs = _specs(3, 5, d, k=4, criterion=2 if is_reg else 0, msl=2)
    T = len(specs)
    # fit 0: +1 / -1 constraints; fit 1: unconstrained row of a constrained build; fit 2: +1 only
    mono = np.zeros((3, d), dtype=np.int8)
    mono[0, :2] = (1, -1)
    mono[2, 0] = 1
    if not is_reg:
        mono = -mono   # classifiers constrain the class-0 fraction (models/forest.py _mono_table)
    tier = forest_ops.ForestTiers(**TIERS[tiers])
    if is_reg:
        g = forest_ops.build_gpu(Xb, None, torch.from_numpy(y).to(dev), torch.from_numpy(roles).to(dev), specs, 1,
                                 True, tier, mono=mono)
        c = forest_ops.build_cpu(Xb_cpu, None, y, roles, specs, 1, True, mono=mono)
    else:
        g = forest_ops.build_gpu(Xb, torch.from_numpy(y).to(dev), None, torch.from_numpy(roles).to(dev), specs, 2,
                                 False, tier, mono=mono)
        c = forest_ops.build_cpu(Xb_cpu, y, None, roles, specs, 2, False, mono=mono)
    gc = _canon(g.nodes.cpu().numpy(), g.vals.cpu().numpy(), T)
    cc = _canon(c.nodes, c.vals, T)
    assert gc == cc


def test_gpu_monotonic_cst_family_matches_host_path():
    """monotonic_cst candidates on device-resident data grow on the HIP builder and score
    exactly what the all-host path scores."""
    from cs230_distributed_machine_learning_amd.data.device import DeviceData
    from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates

    rng = np.random.RandomState(2)
    X = rng.randint(0, 16, size=(3000, 5)).astype(np.float32)
    y = (X[:, 0] - 0.5 * X[:, 1] + 3 * rng.randn(3000) > 4).astype(np.int64)
    cands = [{"n_estimators": 4, "max_depth": 7, "monotonic_cst": c} for c in ([1, -1, 0, 0, 0], None)]
    spec = JobSpec("RandomForestClassifier", cands, cv=3, holdout=False, random_state=1)
    gpu = run_candidates(DeviceData(X, y, True, "cuda:0"), spec, range(len(cands)))
    cpu = run_candidates(DeviceData(X, y, True, "cpu"), spec, range(len(cands)))
    for g, c in zip(gpu, cpu):
        assert g.ok and c.ok
        assert np.allclose(g.result["cv_scores"], c.result["cv_scores"], rtol=0, atol=1e-12)


@pytest.mark.parametrize("is_reg,boot", [(False, 1), (True, 1), (True, 0)])
def test_gpu_whole_histogram_levels_match_cpu(is_reg, boot, monkeypatch):
    """max_features == d (boosting, max_features=None): large-tier levels keep every node's
    histogram over all features and derive the larger of two large siblings as parent -
    smaller sibling (k_hist_derive).  Trees equal the C++ builder's and the row-pass build's
    (DML_LARGE_SUB=0), node for node."""
    from sklearn.datasets import make_regression

    n, d = 40000, 12
    if is_reg:
        X, y = make_regression(n_samples=n, n_features=d, noise=5.0, random_state=2)
        X, y = X.astype(np.float32), (y * 3 + 50).astype(np.float32)
    else:
        X, y = _data(n, d, 3, seed=5)
    dev = torch.device("cuda:0")
    Xb = binning.bin_matrix(torch.from_numpy(X).to(dev), binning.quantile_edges(torch.from_numpy(X).to(dev)))
    roles, _ = make_split_roles(y, 3, not is_reg, holdout=False)
    # boot 0: unit row weights -- the regression large tier keeps u32 row counts in LDS and in
    # the whole-feature buffers (k_hist_large gcnt, whole_counts_u32)
    specs = _specs(3, 4, d, k=d, criterion=2 if is_reg else 0, max_depth=9, bootstrap=boot)
    T = len(specs)
    tiers = forest_ops.ForestTiers(sub_max=64, wave_max=256, block_max=1024, chunk=1024, chunk_reg=1024)
    yt = torch.from_numpy(y).to(dev)
    args = (None, yt, torch.from_numpy(roles).to(dev), specs, 1, True) if is_reg else \
        (yt.to(torch.int32), None, torch.from_numpy(roles).to(dev), specs, 3, False)
    g = forest_ops.build_gpu(Xb, *args, tiers)
    assert g.stats["tier_nodes"][3] > 3 * T   # large-tier levels below the roots
    monkeypatch.setenv("DML_LARGE_SUB", "0")
    g0 = forest_ops.build_gpu(Xb, *args, tiers)
    c = forest_ops.build_cpu(Xb.cpu().numpy(), None if is_reg else y.astype(np.int32), y if is_reg else None, roles,
                             specs, 1 if is_reg else 3, is_reg)
    gc = _canon(g.nodes.cpu().numpy(), g.vals.cpu().numpy(), T)
    assert gc == _canon(c.nodes, c.vals, T)
    assert gc == _canon(g0.nodes.cpu().numpy(), g0.vals.cpu().numpy(), T)


@pytest.mark.parametrize("kw", [
    dict(),                                               # bootstrap, full depth
    dict(msl=3, max_depth=7),
    dict(k=3, mid=0.02),                                  # feature sampling, min_impurity_decrease
    dict(bootstrap=0, mwf=0.01, mss=6),
])
@pytest.mark.parametrize("big_rows", [None, "256"])
def test_gpu_absolute_error_trees_match_cpu(kw, big_rows, monkeypatch):
    """criterion="absolute_error" on the GPU MAE builder (forest_mae.hip): rows in target
    order, exact fixed-point abs deviations -- the host builder's trees node for node
    (splits, medians, abs deviations in the node values).  big_rows=256: nodes of >= 256
    rows take the feature-parallel path (k_mae_eval + k_mae_decide)."""
    if big_rows:
        monkeypatch.setenv("DML_MAE_BIG_ROWS", big_rows)
    rng = np.random.RandomState(7)
    n, d = 6000, 6
    X = rng.randint(0, 20, size=(n, d)).astype(np.float32)
    X[:, 3] = rng.randn(n)                                 # one continuous column
    y = (X[:, 0] - 0.7 * X[:, 1] + 3 * rng.standard_t(2, n)).astype(np.float32)
    y[rng.rand(n) < 0.1] = 0.0                             # repeated targets: median ties
    dev = torch.device("cuda:0")
    Xb = binning.bin_matrix(torch.from_numpy(X).to(dev), binning.quantile_edges(torch.from_numpy(X).to(dev)))
    roles, _ = make_split_roles(y, 3, False, holdout=False)
    specs = _specs(3, 3, d, criterion=forest_ops.MAE, **{k: v for k, v in kw.items() if k != "k"},
                   k=kw.get("k", d))
    T = len(specs)
    g = forest_ops.build_gpu_mae(Xb, torch.from_numpy(y).to(dev), torch.from_numpy(roles).to(dev), specs)
    c = forest_ops.build_cpu(Xb.cpu().numpy(), None, y, roles, specs, 1, True)
    gc = _canon(g.nodes.cpu().numpy(), g.vals.cpu().numpy(), T)
    cc = _canon(c.nodes, c.vals, T)
    assert sum(map(len, gc)) == sum(map(len, cc)) > 10 * T
    assert gc == cc


@pytest.mark.parametrize("extra,seeds", [({}, (1, 3, 6)), ({"max_depth": 4}, (1, 2)),
                                         ({"max_leaf_nodes": 12}, (1, 2)), ({"ccp_alpha": 0.05}, (1, 2))])
def test_gpu_absolute_error_matches_sklearn(extra, seeds):
    """The GPU-grown absolute_error trees against sklearn's (exactly binned columns), the
    same check (and seeds: full-depth trees on other seeds hit equal-gain ties between
    features) tests/test_models_cpu.py makes for the host builder."""
    from sklearn.ensemble import RandomForestRegressor

    from cs230_distributed_machine_learning_amd.data.device import DeviceData
    from cs230_distributed_machine_learning_amd.engine.service import refit_model

    rng = np.random.default_rng(3)
    X = rng.integers(0, 8, size=(400, 4)).astype(np.float32)
    y = np.round((1.5 * X[:, 0] - X[:, 1] + rng.standard_t(2, 400)) * 8) / 8
    for seed in seeds:
        params = {"n_estimators": 1, "bootstrap": False, "max_features": None, "criterion": "absolute_error",
                  "min_samples_leaf": 3, "random_state": seed, **extra}
        m = refit_model({"model_type": "RandomForestRegressor", "scoring": None}, params,
                        DeviceData(X, y, False, "cuda:0"))
        sk = RandomForestRegressor(**params).fit(X, y).estimators_[0].tree_
        nodes, vals = np.asarray(m["nodes"]), np.asarray(m["vals"])
        leaves = nodes[:, 0] < 0
        ours = np.sort(vals[leaves, 1] / vals[leaves, 0])
        ref = np.sort(sk.value[sk.children_left == -1][:, 0, 0])
        assert len(ours) == len(ref)
        np.testing.assert_allclose(ours, ref, rtol=1e-9)


def test_gpu_block_tier_settings_do_not_change_trees(monkeypatch):
    """Round 6 block-tier settings (2-wave binary nodes, kg_block = the batch's largest
    max_features, binary wave_max 256) against the round-5 ones (kg_block 16, wave_max 512):
    the same trees, node for node -- feature groups and tier thresholds never change a tree."""
    n, d, C = 120_000, 24, 2
    X, y = _data(n, d, C, seed=3)
    dev = torch.device("cuda:0")
    edges = binning.quantile_edges(torch.from_numpy(X))
    Xb_cpu = binning.bin_matrix(torch.from_numpy(X), edges).numpy()
    Xb = torch.from_numpy(Xb_cpu).to(dev)
    roles, _ = make_split_roles(y, 3, True, holdout=False)
    specs = _specs(3, 4, d, msl=2)
    specs["max_features"][:4] = 5      # a batch of mixed max_features: kg_block = 9 here
    specs["max_features"][4:8] = 9
    ycls = torch.from_numpy(y.astype(np.int32)).to(dev)
    rl = torch.from_numpy(roles).to(dev)
    builds = {}
    for name, env in (("auto", {}), ("r5", {"DML_TIER_KG_BLOCK": "16", "DML_TIER_WAVE_MAX": "512"})):
        for k in ("DML_TIER_KG_BLOCK", "DML_TIER_WAVE_MAX"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        g = forest_ops.build_gpu(Xb, ycls, None, rl, specs, C, False, forest_ops.ForestTiers())
        assert g.stats["tier_nodes"][2] > 0   # the block tier ran
        builds[name] = _canon(g.nodes.cpu().numpy(), g.vals.cpu().numpy(), len(specs))
    assert builds["auto"] == builds["r5"]
    c = forest_ops.build_cpu(Xb_cpu, y.astype(np.int32), None, roles, specs, C, False)
    assert builds["auto"] == _canon(c.nodes, c.vals, len(specs))


@pytest.mark.parametrize("n_fits,msl,depth", [(3, 1, 14), (2, 4, 2**31 - 1)])
def test_gpu_row_window_path_matches_cpu(n_fits, msl, depth):
    """d = 100 on 128-byte rows (the engine's padded layout, ops/binning.py row_pitch): the block
    tier's first feature group and the wave tier's prefetch read whole row lines (dwordx4
    windows) -- the bench's path, node for node against the C++ builder."""
    n, d, C = 80_000, 100, 2
    X, y = _data(n, d, C, seed=11)
    dev = torch.device("cuda:0")
    edges = binning.quantile_edges(torch.from_numpy(X))
    Xb_cpu = binning.bin_matrix(torch.from_numpy(X), edges).numpy()
    pad = torch.zeros((n, 128), dtype=torch.uint8, device=dev)
    pad[:, :d] = torch.from_numpy(Xb_cpu).to(dev)
    Xb = pad[:, :d]
    assert Xb.stride(0) == 128
    roles, _ = make_split_roles(y, n_fits, True, holdout=False)
    specs = _specs(n_fits, 3, d, msl=msl, max_depth=depth)   # max_features sqrt(100) = 10
    ycls = y.astype(np.int32)
    g = forest_ops.build_gpu(Xb, torch.from_numpy(ycls).to(dev), None, torch.from_numpy(roles).to(dev), specs, C,
                             False, forest_ops.ForestTiers())
    assert g.stats["tier_nodes"][1] > 0 and g.stats["tier_nodes"][2] > 0   # wave and block tiers ran
    c = forest_ops.build_cpu(Xb_cpu, ycls, None, roles, specs, C, False)
    assert _canon(g.nodes.cpu().numpy(), g.vals.cpu().numpy(), len(specs)) == _canon(c.nodes, c.vals, len(specs))
