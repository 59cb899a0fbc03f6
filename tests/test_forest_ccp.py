"""RandomForest ``ccp_alpha``: minimal cost-complexity pruning (ops/forest_ops.py prune_ccp).

The bottom-up pass must keep exactly the subtree that sklearn's weakest-link loop
(``_cost_complexity_prune``: prune the smallest effective alpha while it is <= ccp_alpha)
ends with.  The reference below is that loop, written out in numpy over our own trees."""
import numpy as np
import pytest
import torch

from cs230_distributed_machine_learning_amd.models.forest import native_seed
from cs230_distributed_machine_learning_amd.ops import binning, forest_ops
from cs230_distributed_machine_learning_amd.utils import native


def _imp(v, is_reg, crit):
    if is_reg:
        return (v[0], v[2] / v[0] - (v[1] / v[0]) ** 2) if v[0] > 0 else (0.0, 0.0)
    w = v.sum()
    p = v / w
    if crit == forest_ops.ENTROPY:
        return w, float(-(p[p > 0] * np.log2(p[p > 0])).sum())
    return w, float(1.0 - (p * p).sum())


def _weakest_link(nodes, vals, root, alpha, is_reg, crit):
    """sklearn's loop: returns the set of internal nodes that survive."""
    nodes = nodes.copy()
    W = _imp(vals[root], is_reg, crit)[0]
    R = {}

    def reach(t):
        out = [t]
        if nodes[t, 0] >= 0:
            out += reach(nodes[t, 1]) + reach(nodes[t, 1] + 1)
        return out

    while True:
        best, best_g = None, np.inf
        for t in reach(root):
            if nodes[t, 0] < 0:
                continue
            sub = reach(t)
            lv = [u for u in sub if nodes[u, 0] < 0]
            for u in [t] + lv:
                if u not in R:
                    w, im = _imp(vals[u], is_reg, crit)
                    R[u] = w / W * im
            g = (R[t] - sum(R[u] for u in lv)) / (len(lv) - 1)
            if g < best_g:
                best, best_g = t, g
        if best is None or best_g > alpha:
            break
        nodes[best] = (-1, -1)
    return {t for t in reach(root) if nodes[t, 0] >= 0}


@pytest.mark.parametrize("is_reg,crit", [(False, forest_ops.GINI), (False, forest_ops.ENTROPY), (True, forest_ops.MSE)])
def test_ccp_matches_weakest_link_loop(is_reg, crit):
    rng = np.random.default_rng(4)
    n, d = 600, 6
    X = rng.normal(size=(n, d)).astype(np.float32)
    y = (X[:, 0] + 0.8 * rng.normal(size=n) > 0).astype(np.int32) + (X[:, 1] > 0.7)
    yr = (X[:, 0] + 0.5 * rng.normal(size=n)).astype(np.float32)
    Xb = binning.bin_matrix(torch.from_numpy(X), binning.quantile_edges(torch.from_numpy(X))).numpy()
    T = 4
    specs = forest_ops.make_specs(T)
    specs["seed"] = [native_seed(9, j) for j in range(T)]
    specs["max_depth"], specs["min_samples_split"], specs["min_samples_leaf"] = 2**31 - 1, 2, 1
    specs["max_features"], specs["bootstrap"], specs["criterion"] = d, 1, crit
    specs["pois_cdf"] = native.poisson_cdf_table(1.0)
    roles = np.ones((1, n), np.uint8)
    C = 1 if is_reg else 3
    fb = forest_ops.build_cpu(Xb, None if is_reg else y, yr if is_reg else None, roles, specs, C, is_reg)
    alphas = np.array([0.002, 0.01, 0.0, 0.03])
    ref = [_weakest_link(fb.nodes, fb.vals, t, a, is_reg, crit) if a > 0 else None for t, a in enumerate(alphas)]
    before = fb.nodes.copy()
    leaves = forest_ops.prune_ccp(fb, specs, alphas)

    def internal(t):
        out, st = set(), [t]
        while st:
            u = st.pop()
            if fb.nodes[u, 0] >= 0:
                out.add(u)
                st += [fb.nodes[u, 1], fb.nodes[u, 1] + 1]
        return out

    for t in range(T):
        if alphas[t] == 0:
            assert np.array_equal(before[t], fb.nodes[t])
            continue
        assert internal(t) == ref[t], t
        assert leaves[t] == len(ref[t]) + 1
    assert leaves[1] < leaves[0] or leaves[0] == 1


def test_ccp_alpha_through_the_family_prunes_like_sklearn():
    """A job grid over ccp_alpha: larger alphas give fewer leaves, and on a table where our
    splits are sklearn's (exactly binned integer columns, no bootstrap, all features) the
    pruned tree keeps the same leaf count as sklearn's."""
    from sklearn.ensemble import RandomForestClassifier

    from cs230_distributed_machine_learning_amd.data.device import DeviceData
    from cs230_distributed_machine_learning_amd.engine.service import refit_model

    rng = np.random.default_rng(0)
    X = rng.integers(0, 6, size=(400, 3)).astype(np.float32)
    y = ((X[:, 0] + X[:, 1] + rng.integers(0, 3, 400)) > 6).astype(np.int64)
    grid = [{"n_estimators": 1, "bootstrap": False, "max_features": None, "ccp_alpha": a, "random_state": 0}
            for a in (0.0, 0.005, 0.02)]
    ours = []
    for g in grid:   # refit: one fit on every row (engine/service.py refit_model)
        m = refit_model({"model_type": "RandomForestClassifier", "scoring": None}, g, DeviceData(X, y, True))
        ours.append(int((np.asarray(m["nodes"])[:, 0] < 0).sum()))
    assert ours[0] > ours[1] >= ours[2]
    for g, got in zip(grid, ours):
        sk = RandomForestClassifier(**g).fit(X, y)
        assert got == sk.estimators_[0].get_n_leaves(), (g, got, sk.estimators_[0].get_n_leaves())


@pytest.mark.parametrize("model", ["GradientBoostingRegressor", "GradientBoostingClassifier"])
def test_gbrt_ccp_alpha_matches_sklearn(model):
    """Each stage tree is pruned before its leaf values are set, as sklearn's trees are."""
    from sklearn import ensemble
    from sklearn.datasets import make_classification, make_regression

    from cs230_distributed_machine_learning_amd.data.device import DeviceData
    from cs230_distributed_machine_learning_amd.models.base import FitTask, family_of
    from cs230_distributed_machine_learning_amd.models.boosting import gbrt_raw_numpy

    reg = model.endswith("Regressor")
    if reg:
        X, y = make_regression(300, 4, noise=10, random_state=2)
        y = np.round(y, 2)
        ccp = 20.0
    else:
        X, y = make_classification(300, 5, n_informative=4, n_redundant=0, random_state=3)
        ccp = 0.002
    X = np.round(X, 1)
    params = {"n_estimators": 6, "max_depth": 4, "ccp_alpha": ccp}
    sk = getattr(ensemble, model)(random_state=0, **params).fit(X, y)
    ref = sk.predict(X) if reg else sk.decision_function(X)
    dd = DeviceData(X, y, not reg, "cpu")
    dd.set_splits(np.ones((1, len(y)), np.uint8), ["full"])
    fam = family_of(model)
    rp = fam.resolve(model, params, len(y), X.shape[1], 1 if reg else 2)
    out = fam.run(dd, [FitTask(0, 0, 0, model, rp)], keep_models=True)[0]
    got = gbrt_raw_numpy(out.model, X)[:, 0]
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-3)
    pruned = sum(e[0].get_n_leaves() for e in sk.estimators_)
    full = sum(e[0].get_n_leaves() for e in getattr(ensemble, model)(
        random_state=0, n_estimators=6, max_depth=4).fit(X, y).estimators_)
    assert pruned < full      # the alpha really prunes


@pytest.mark.gpu
def test_ccp_on_device_matches_host():
    rng = np.random.default_rng(5)
    n, d = 20000, 10
    X = rng.normal(size=(n, d)).astype(np.float32)
    y = (X[:, 0] + 0.8 * rng.normal(size=n) > 0).astype(np.int32)
    dev = torch.device("cuda:0")
    Xt = torch.from_numpy(X)
    E = binning.quantile_edges(Xt)
    Xb = binning.bin_matrix(Xt, E).numpy()
    Xg = binning.bin_matrix(Xt.to(dev), E.to(dev))
    T = 6
    specs = forest_ops.make_specs(T)
    specs["seed"] = [native_seed(2, j) for j in range(T)]
    specs["max_depth"], specs["min_samples_split"], specs["min_samples_leaf"] = 2**31 - 1, 2, 1
    specs["max_features"], specs["bootstrap"], specs["criterion"] = 3, 1, forest_ops.GINI
    specs["pois_cdf"] = native.poisson_cdf_table(1.0)
    roles = np.ones((1, n), np.uint8)
    alphas = np.array([1e-4, 5e-4, 0.0, 2e-3, 1e-5, 1e-3])
    host = forest_ops.build_cpu(Xb, y, None, roles, specs, 2, False)
    gpu = forest_ops.build_gpu(Xg, torch.from_numpy(y).to(dev), None, torch.from_numpy(roles).to(dev), specs, 2, False)
    lh = forest_ops.prune_ccp(host, specs, alphas)
    lg = forest_ops.prune_ccp(gpu, specs, alphas)
    assert np.array_equal(lh, lg)
    rows = np.arange(n, dtype=np.int32)
    toff, roff = np.array([0, T]), np.array([0, n])
    ph = forest_ops.predict(host, Xb, toff, roff, rows)
    pg = forest_ops.predict(gpu, Xg, toff, roff, torch.from_numpy(rows).to(dev)).cpu().numpy()
    assert np.array_equal(ph, pg)
