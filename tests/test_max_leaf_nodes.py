"""max_leaf_nodes for RandomForest* and GradientBoosting* vs sklearn.

sklearn grows a tree with max_leaf_nodes best-first (expand the frontier node of largest
impurity improvement, L-1 expansions); the builders grow the tree depth-first and cut it
to exactly that best-first top (csrc/kernels/forest_common.h best_first_prune; the split
at every node depends only on that node).  With every feature exactly binned the fitted
functions are sklearn's."""
import numpy as np
import pytest

from cs230_distributed_machine_learning_amd.data.device import DeviceData
from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates
from cs230_distributed_machine_learning_amd.models.base import FitTask, family_of
from cs230_distributed_machine_learning_amd.search.grid import ParameterGrid

sk = pytest.importorskip("sklearn")
from sklearn.datasets import make_classification, make_regression  # noqa: E402
from sklearn.model_selection import GridSearchCV  # noqa: E402


def _count_leaves(nodes, root):
    stack, leaves = [root], 0
    while stack:
        i = stack.pop()
        if nodes[i, 0] < 0:
            leaves += 1
        else:
            stack += [nodes[i, 1], nodes[i, 1] + 1]
    return leaves


@pytest.mark.parametrize("L", [2, 5, 13])
def test_gbrt_regressor_max_leaf_nodes_full_fit_matches_sklearn(L):
    from sklearn.ensemble import GradientBoostingRegressor

    from cs230_distributed_machine_learning_amd.models.boosting import gbrt_raw_numpy

    X, y = make_regression(400, 5, noise=10, random_state=7)
    X, y = np.round(X, 1), np.round(y, 2)
    params = {"n_estimators": 6, "max_leaf_nodes": L, "max_depth": None, "learning_rate": 0.2}
    ref = GradientBoostingRegressor(random_state=0, **params).fit(X, y).predict(X)
    dd = DeviceData(X, y, False, "cpu")
    dd.set_splits(np.ones((1, len(y)), np.uint8), ["full"])
    fam = family_of("GradientBoostingRegressor")
    rp = fam.resolve("GradientBoostingRegressor", params, len(y), X.shape[1], 1)
    out = fam.run(dd, [FitTask(0, 0, 0, "GradientBoostingRegressor", rp)], keep_models=True)[0]
    assert not out.info.get("warnings")
    np.testing.assert_allclose(gbrt_raw_numpy(out.model, X)[:, 0], ref, rtol=1e-4, atol=1e-3)


def test_gbrt_classifier_max_leaf_nodes_full_fit_matches_sklearn():
    from sklearn.ensemble import GradientBoostingClassifier

    from cs230_distributed_machine_learning_amd.models.boosting import gbrt_raw_numpy

    X, y = make_classification(300, 5, n_informative=4, n_redundant=0, n_classes=3, random_state=3)
    X = np.round(X, 1)
    params = {"n_estimators": 5, "max_leaf_nodes": 6, "learning_rate": 0.3}
    ref = GradientBoostingClassifier(random_state=0, **params).fit(X, y).decision_function(X)
    dd = DeviceData(X, y, True, "cpu")
    dd.set_splits(np.ones((1, len(y)), np.uint8), ["full"])
    fam = family_of("GradientBoostingClassifier")
    rp = fam.resolve("GradientBoostingClassifier", params, len(y), X.shape[1], 3)
    out = fam.run(dd, [FitTask(0, 0, 0, "GradientBoostingClassifier", rp)], keep_models=True)[0]
    np.testing.assert_allclose(gbrt_raw_numpy(out.model, X), ref, atol=1e-9)


def test_rf_single_tree_max_leaf_nodes_matches_sklearn_cv():
    """No bootstrap, every feature: each tree is sklearn's best-first tree -> equal CV scores."""
    from sklearn.ensemble import RandomForestClassifier, RandomForestRegressor

    X, y = make_classification(600, 6, n_informative=5, n_redundant=0, n_classes=3, random_state=11)
    X = np.round(X, 1)
    grid = {"max_leaf_nodes": [2, 4, 9, 25], "n_estimators": [1], "bootstrap": [False], "max_features": [None]}
    dd = DeviceData(X, y, True, "cpu")
    res = run_candidates(dd, JobSpec("RandomForestClassifier", list(ParameterGrid(grid)), cv=5), range(4))
    ours = np.array([r.result["mean_cv_score"] for r in res])
    ref = GridSearchCV(RandomForestClassifier(random_state=0), grid, cv=5).fit(X, y).cv_results_["mean_test_score"]
    np.testing.assert_allclose(ours, ref, atol=1e-12)

    Xr, yr = make_regression(500, 5, noise=5, random_state=12)
    Xr, yr = np.round(Xr, 1), np.round(yr, 2)
    dr = DeviceData(Xr, yr, False, "cpu")
    res = run_candidates(dr, JobSpec("RandomForestRegressor", list(ParameterGrid(grid)), cv=5), range(4))
    ours = np.array([r.result["mean_cv_score"] for r in res])
    ref = GridSearchCV(RandomForestRegressor(random_state=0), grid, cv=5).fit(Xr, yr).cv_results_["mean_test_score"]
    # regression: near-equal improvements of two frontier nodes can order differently
    # (sklearn's running sums vs our per-node sums round differently) -> one late leaf
    np.testing.assert_allclose(ours[:3], ref[:3], atol=1e-9)
    assert abs(ours[3] - ref[3]) < 2e-3


def test_rf_max_leaf_nodes_bounds_every_tree_and_tracks_sklearn():
    from sklearn.ensemble import RandomForestClassifier

    X, y = make_classification(3000, 12, n_informative=6, random_state=5)
    X = X.astype(np.float32)
    grid = {"max_leaf_nodes": [8, 64], "n_estimators": [40]}
    dd = DeviceData(X, y, True, "cpu")
    res = run_candidates(dd, JobSpec("RandomForestClassifier", list(ParameterGrid(grid)), cv=3, keep_models="all"),
                         range(2))
    ref = GridSearchCV(RandomForestClassifier(random_state=0), grid, cv=3).fit(X, y).cv_results_["mean_test_score"]
    ours = np.array([r.result["mean_cv_score"] for r in res])
    assert np.abs(ours - ref).max() < 0.02, (ours, ref)
    for r, L in zip(res, (8, 64)):
        m = r.model
        leaves = [_count_leaves(m["nodes"], t) for t in range(m["n_trees"])]
        assert max(leaves) <= L and min(leaves) >= L // 2, leaves


def test_max_leaf_nodes_validation():
    fam = family_of("RandomForestClassifier")
    with pytest.raises(Exception):
        fam.resolve("RandomForestClassifier", {"max_leaf_nodes": 1}, 100, 4, 2)
    rp = fam.resolve("RandomForestClassifier", {"max_leaf_nodes": None}, 100, 4, 2)
    assert rp["max_leaf_nodes"] == 0 and not rp["warnings"]
