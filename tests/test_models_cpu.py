"""Estimator families on CPU vs scikit-learn (reference whitelist worker.py:36-57)."""
import numpy as np
import pytest

from cs230_distributed_machine_learning_amd.data.device import DeviceData
from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates
from cs230_distributed_machine_learning_amd.models.base import FitTask, family_of
from cs230_distributed_machine_learning_amd.search.grid import ParameterGrid

sk = pytest.importorskip("sklearn")
from sklearn.datasets import load_iris, make_classification, make_regression  # noqa: E402
from sklearn.model_selection import GridSearchCV  # noqa: E402


def _ours(model, X, y, clf, grid, cv=5):
    dd = DeviceData(X, y, clf, "cpu")
    cands = list(ParameterGrid(grid))
    res = run_candidates(dd, JobSpec(model, cands, cv=cv), range(len(cands)))
    assert all(r.ok for r in res), [r.error for r in res if not r.ok]
    return np.array([r.result["mean_cv_score"] for r in res])


def _ref(est, X, y, grid, cv=5):
    return GridSearchCV(est, grid, cv=cv).fit(X, y).cv_results_["mean_test_score"]


def test_knn_classifier_matches_sklearn():
    from sklearn.neighbors import KNeighborsClassifier

    X, y = make_classification(600, 8, n_informative=5, n_classes=3, random_state=0)
    grid = {"n_neighbors": [1, 3, 7, 15], "weights": ["uniform", "distance"], "p": [1, 2, 3]}
    np.testing.assert_allclose(_ours("KNeighborsClassifier", X, y, True, grid),
                               _ref(KNeighborsClassifier(), X, y, grid), atol=1e-12)


def test_knn_regressor_matches_sklearn():
    from sklearn.neighbors import KNeighborsRegressor

    X, y = make_regression(500, 6, noise=5, random_state=1)
    grid = {"n_neighbors": [2, 5, 9], "weights": ["uniform", "distance"], "metric": ["euclidean", "manhattan",
                                                                                      "chebyshev"]}
    np.testing.assert_allclose(_ours("KNeighborsRegressor", X, y, False, grid),
                               _ref(KNeighborsRegressor(), X, y, grid), atol=1e-6)


def test_knn_too_many_neighbors_is_a_failed_candidate():
    X, y = load_iris(return_X_y=True)
    dd = DeviceData(X, y, True, "cpu")
    res = run_candidates(dd, JobSpec("KNeighborsClassifier", [{"n_neighbors": 500}, {"n_neighbors": 3}], cv=5),
                         [0, 1])
    assert not res[0].ok and "n_neighbors" in res[0].error
    assert res[1].ok


@pytest.mark.parametrize("loss,n_classes", [("log_loss", 2), ("exponential", 2), ("log_loss", 3)])
def test_gbrt_classifier_full_fit_matches_sklearn(loss, n_classes):
    """With every feature exactly binned, a GBRT fit reproduces sklearn's raw scores."""
    from sklearn.ensemble import GradientBoostingClassifier

    from cs230_distributed_machine_learning_amd.models.boosting import gbrt_raw_numpy

    X, y = make_classification(300, 5, n_informative=4, n_redundant=0, n_classes=n_classes, random_state=3)
    X = np.round(X, 1)
    params = {"n_estimators": 8, "loss": loss, "max_depth": 2, "learning_rate": 0.3}
    ref = GradientBoostingClassifier(random_state=0, **params).fit(X, y).decision_function(X)
    dd = DeviceData(X, y, True, "cpu")
    dd.set_splits(np.ones((1, len(y)), np.uint8), ["full"])
    fam = family_of("GradientBoostingClassifier")
    rp = fam.resolve("GradientBoostingClassifier", params, len(y), X.shape[1], n_classes)
    out = fam.run(dd, [FitTask(0, 0, 0, "GradientBoostingClassifier", rp)], keep_models=True)[0]
    raw = gbrt_raw_numpy(out.model, X)
    raw = raw[:, 0] if ref.ndim == 1 else raw
    np.testing.assert_allclose(raw, ref, atol=1e-9)


@pytest.mark.parametrize("loss", ["squared_error", "absolute_error", "huber", "quantile"])
def test_gbrt_regressor_full_fit_matches_sklearn(loss):
    from sklearn.ensemble import GradientBoostingRegressor

    from cs230_distributed_machine_learning_amd.models.boosting import gbrt_raw_numpy

    X, y = make_regression(300, 4, noise=10, random_state=2)
    X = np.round(X, 1)
    y = np.round(y, 2)
    params = {"n_estimators": 6, "loss": loss, "max_depth": 2}
    ref = GradientBoostingRegressor(random_state=0, **params).fit(X, y).predict(X)
    dd = DeviceData(X, y, False, "cpu")
    dd.set_splits(np.ones((1, len(y)), np.uint8), ["full"])
    fam = family_of("GradientBoostingRegressor")
    rp = fam.resolve("GradientBoostingRegressor", params, len(y), X.shape[1], 1)
    out = fam.run(dd, [FitTask(0, 0, 0, "GradientBoostingRegressor", rp)], keep_models=True)[0]
    got = gbrt_raw_numpy(out.model, X)[:, 0]
    if loss == "quantile":
        # quantile pseudo-residuals take two values, so many splits tie on gain: which of
        # the tied splits wins depends on the feature visiting order (sklearn's RNG vs
        # ours), not on the model -- the fits agree except on a handful of rows
        close = np.isclose(got, ref, rtol=1e-4, atol=1e-3)
        assert close.mean() >= 0.97, close.mean()
    else:
        np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-3)


def test_gbrt_grid_close_to_sklearn():
    from sklearn.ensemble import GradientBoostingClassifier

    X, y = make_classification(400, 6, n_informative=4, random_state=0)
    X = np.round(X, 1)
    grid = {"n_estimators": [20, 50], "learning_rate": [0.1, 0.5]}
    ours = _ours("GradientBoostingClassifier", X, y, True, grid)
    ref = _ref(GradientBoostingClassifier(random_state=0), X, y, grid)
    # exact-value bins + sklearn midpoint thresholds: only equal-gain feature ties differ
    assert np.abs(ours - ref).max() < 0.01


def test_gbrt_subsample_runs():
    X, y = make_regression(300, 4, noise=10, random_state=2)
    s = _ours("GradientBoostingRegressor", X, y, False, {"subsample": [0.5], "n_estimators": [30],
                                                          "random_state": [0]})
    assert s[0] > 0.5


def test_logistic_matches_sklearn_iris():
    from sklearn.linear_model import LogisticRegression

    X, y = load_iris(return_X_y=True)
    # the reference demo grid; C=10/100 lbfgs stop at max_iter=100 unconverged, and the
    # host L-BFGS-B path still reproduces sklearn's iterates
    grid = {"C": [0.1, 1.0, 10.0, 100], "solver": ["lbfgs"]}
    np.testing.assert_allclose(_ours("LogisticRegression", X, y, True, grid),
                               _ref(LogisticRegression(), X, y, grid), atol=1e-12)
    grid = {"C": [0.01, 0.1, 1.0], "solver": ["liblinear"]}
    assert np.abs(_ours("LogisticRegression", X, y, True, grid) -
                  _ref(LogisticRegression(), X, y, grid)).max() <= 0.0134


def test_random_forest_close_to_sklearn():
    from sklearn.ensemble import RandomForestClassifier

    X, y = make_classification(500, 8, n_informative=5, random_state=4)
    grid = {"n_estimators": [50], "max_depth": [3, None]}
    ours = _ours("RandomForestClassifier", X, y, True, grid)
    ref = _ref(RandomForestClassifier(random_state=0), X, y, grid)
    assert np.abs(ours - ref).max() < 0.05


def test_unsupported_model_is_rejected():
    from cs230_distributed_machine_learning_amd.models.base import ParamError

    with pytest.raises(ParamError):
        family_of("MLPClassifier")


def test_svc_matches_sklearn_iris():
    from sklearn.svm import SVC

    X, y = load_iris(return_X_y=True)
    grid = {"C": [0.1, 1, 10], "kernel": ["rbf", "linear", "poly", "sigmoid"]}
    np.testing.assert_allclose(_ours("SVC", X, y, True, grid), _ref(SVC(), X, y, grid), atol=1e-12)


def test_svc_binary_class_weight_matches_sklearn():
    from sklearn.svm import SVC

    X, y = make_classification(300, 6, n_informative=4, weights=[0.7], random_state=0)
    grid = {"C": [0.5, 5], "gamma": ["scale", 0.05], "class_weight": [None, "balanced"]}
    np.testing.assert_allclose(_ours("SVC", X, y, True, grid), _ref(SVC(), X, y, grid), atol=1e-12)


def test_svr_matches_sklearn():
    from sklearn.svm import SVR

    X, y = make_regression(200, 4, noise=10, random_state=2)
    y = y / 50
    grid = {"C": [1, 10], "epsilon": [0.05, 0.2], "kernel": ["rbf", "linear"]}
    np.testing.assert_allclose(_ours("SVR", X, y, False, grid), _ref(SVR(), X, y, grid), atol=1e-4)


def test_saved_models_predict_like_training(tmp_path):
    """refit artefacts (.npz, no pickle) of every family predict on the host."""
    from cs230_distributed_machine_learning_amd.engine.model_store import load_model, predict, save_model

    X, y = load_iris(return_X_y=True)
    for model, params in [("SVC", {"C": 3.0}), ("KNeighborsClassifier", {"n_neighbors": 3}),
                          ("GradientBoostingClassifier", {"n_estimators": 5}),
                          ("RandomForestClassifier", {"n_estimators": 5, "random_state": 0}),
                          ("LogisticRegression", {"C": 1.0})]:
        dd = DeviceData(X, y, True, "cpu")
        dd.set_splits(np.ones((1, len(y)), np.uint8), ["full"])
        fam = family_of(model)
        rp = fam.resolve(model, params, len(y), 4, 3)
        out = fam.run(dd, [FitTask(0, 0, 0, model, rp)], keep_models=True)[0]
        path = save_model(out.model, str(tmp_path / f"{model}.npz"))
        pred = predict(load_model(path), X)
        assert (np.asarray(pred).astype(int) == y).mean() > 0.9, model


@pytest.mark.parametrize("grid", [{"n_components": [1, 2, 3, 4]}, {"n_components": [0.9, 0.99, "mle", None]},
                                  {"n_components": [2, 3], "whiten": [True]}])
def test_pca_cv_log_likelihood_matches_sklearn(grid):
    from sklearn.decomposition import PCA

    rng = np.random.RandomState(0)
    X = rng.randn(300, 6) @ rng.randn(6, 6) + rng.randn(300, 6) * 0.1
    y = rng.randint(0, 2, 300)
    dd = DeviceData(X, y, False, "cpu")
    cands = list(ParameterGrid(grid))
    res = run_candidates(dd, JobSpec("PCA", cands, cv=5), range(len(cands)))
    assert all(r.ok for r in res), [r.error for r in res]
    ours = np.array([r.result["mean_cv_score"] for r in res])
    ref = GridSearchCV(PCA(), grid, cv=5).fit(X).cv_results_["mean_test_score"]
    np.testing.assert_allclose(ours, ref, rtol=1e-5)


def test_column_transformers_are_rejected_with_guidance():
    X, y = load_iris(return_X_y=True)
    dd = DeviceData(X, y, True, "cpu")
    res = run_candidates(dd, JobSpec("StandardScaler", [{}], cv=3), [0])
    assert not res[0].ok and "/preprocess" in res[0].error


def test_logistic_l1_and_elasticnet_close_to_sklearn():
    """OWL-QN on the device solver reaches sklearn's liblinear / saga optima."""
    from sklearn.linear_model import LogisticRegression

    X, y = make_classification(1500, 20, n_informative=6, random_state=0)
    for grid in ({"C": [0.01, 0.1, 1.0], "penalty": ["l1"], "solver": ["liblinear", "saga"]},
                 {"C": [0.05, 1.0], "penalty": ["elasticnet"], "solver": ["saga"], "l1_ratio": [0.2, 0.8]}):
        ours = _ours("LogisticRegression", X, y, True, grid)
        ref = _ref(LogisticRegression(max_iter=3000), X, y, grid)
        assert np.abs(ours - ref).max() <= 0.004, (grid, ours, ref)


def test_logistic_class_weight_matches_sklearn():
    from sklearn.linear_model import LogisticRegression

    X, y = make_classification(3000, 10, weights=[0.85], random_state=1)
    for grid in ({"C": [0.1, 1.0], "class_weight": [None, "balanced", {0: 3.0, 1: 1.0}]},
                 {"C": [0.1], "class_weight": ["balanced"], "solver": ["liblinear", "saga"]}):
        np.testing.assert_allclose(_ours("LogisticRegression", X, y, True, grid),
                                   _ref(LogisticRegression(max_iter=3000), X, y, grid), atol=1e-3)


def test_rf_friedman_mse_is_squared_error_split_for_split():
    """friedman_mse's proxy is W_node x (squared-error proxy - const): same trees, no warning."""
    from sklearn.datasets import make_regression

    X, y = make_regression(400, 6, noise=5, random_state=1)
    fam = family_of("RandomForestRegressor")
    outs = []
    for crit in ("squared_error", "friedman_mse"):
        dd = DeviceData(X, y, False, "cpu")
        dd.set_splits(np.ones((1, len(y)), np.uint8), ["full"])
        rp = fam.resolve("RandomForestRegressor", {"criterion": crit, "n_estimators": 5, "random_state": 3},
                         len(y), X.shape[1], 1)
        assert rp["warnings"] == []
        o = fam.run(dd, [FitTask(0, 0, 0, "RandomForestRegressor", rp)], keep_models=True)[0]
        outs.append(o.model)
    assert np.array_equal(outs[0]["nodes"], outs[1]["nodes"])


@pytest.mark.parametrize("mid", [0.5, 2.0, 8.0])
def test_friedman_mse_min_impurity_decrease_matches_sklearn(mid):
    """min_impurity_decrease under friedman_mse reads sklearn's FriedmanMSE improvement
    (w_r s_l - w_l s_r)^2 / (w_l w_r W_node), not the tree-weight-scaled squared-error one
    (forest_common.h accept_improvement): sklearn's trees for both criteria."""
    from sklearn.ensemble import GradientBoostingRegressor, RandomForestRegressor

    from cs230_distributed_machine_learning_amd.engine.service import refit_model

    rng = np.random.default_rng(3)
    X = rng.integers(0, 8, size=(500, 4)).astype(np.float32)
    y = np.round((0.5 * X[:, 0] - 0.3 * X[:, 1] + np.sin(X[:, 2]) + rng.standard_normal(500)) * 8) / 8
    for crit in ("friedman_mse", "squared_error"):
        params = {"n_estimators": 1, "bootstrap": False, "max_features": None, "criterion": crit,
                  "min_impurity_decrease": mid, "random_state": 1}
        m = refit_model({"model_type": "RandomForestRegressor", "scoring": None}, params, DeviceData(X, y, False))
        sk = RandomForestRegressor(**params).fit(X, y).estimators_[0].tree_
        nodes, vals = np.asarray(m["nodes"]), np.asarray(m["vals"])
        lv = nodes[:, 0] < 0
        ref = np.sort(sk.value[sk.children_left == -1][:, 0, 0])
        assert lv.sum() == len(ref)
        np.testing.assert_allclose(np.sort(vals[lv, 1] / vals[lv, 0]), ref, rtol=1e-9)
    # GradientBoosting's default criterion is friedman_mse: the same leaf counts per stage
    params = {"n_estimators": 3, "max_depth": None, "min_impurity_decrease": mid / 4, "random_state": 0}
    m = refit_model({"model_type": "GradientBoostingRegressor", "scoring": None}, params, DeviceData(X, y, False))
    sk = GradientBoostingRegressor(**params).fit(X, y)
    Xq = X[:50].astype(np.float64)
    from cs230_distributed_machine_learning_amd.models.boosting import gbrt_predict_numpy

    np.testing.assert_allclose(gbrt_predict_numpy(m, Xq), sk.predict(Xq), rtol=1e-5, atol=1e-4)


def test_rf_poisson_criterion_matches_sklearn():
    """criterion='poisson': sklearn's proxy (sum_l log mean_l + sum_r log mean_r); on
    exactly binned columns, no bootstrap and every feature, the tree is sklearn's."""
    from sklearn.ensemble import RandomForestRegressor

    from cs230_distributed_machine_learning_amd.engine.service import refit_model

    rng = np.random.default_rng(2)
    X = rng.integers(0, 8, size=(500, 4)).astype(np.float32)
    y = rng.poisson(np.exp(0.3 * X[:, 0] - 0.2 * X[:, 1])).astype(np.float64)
    # equal-gain ties between features go by the visiting order (sklearn's RNG vs our keyed
    # order: squared_error trees differ from sklearn's on some seeds for the same reason);
    # these seeds have no such tie
    for seed in (1, 2):
        params = {"n_estimators": 1, "bootstrap": False, "max_features": None, "criterion": "poisson",
                  "min_samples_leaf": 5, "random_state": seed}
        m = refit_model({"model_type": "RandomForestRegressor", "scoring": None}, params, DeviceData(X, y, False))
        sk = RandomForestRegressor(**params).fit(X, y).estimators_[0].tree_
        nodes, vals = np.asarray(m["nodes"]), np.asarray(m["vals"])
        leaves = nodes[:, 0] < 0
        ours = np.sort(vals[leaves, 1] / vals[leaves, 0])
        ref = np.sort(sk.value[sk.children_left == -1][:, 0, 0])
        assert len(ours) == len(ref)
        np.testing.assert_allclose(ours, ref, rtol=1e-9)
    # ...and it is a different tree from squared_error's
    m2 = refit_model({"model_type": "RandomForestRegressor", "scoring": None}, dict(params, criterion="squared_error"),
                     DeviceData(X, y, False))
    assert not np.array_equal(np.asarray(m2["nodes"]), nodes)
    # negative targets are refused like sklearn
    fam = family_of("RandomForestRegressor")
    rp = fam.resolve("RandomForestRegressor", params, 500, 4, 1)
    dd = DeviceData(X, y - 3.0, False, "cpu")
    dd.set_splits(np.ones((1, len(y)), np.uint8), ["full"])
    with pytest.raises(Exception, match="negative"):
        fam.run(dd, [FitTask(0, 0, 0, "RandomForestRegressor", rp)])


@pytest.mark.parametrize("extra,seeds", [({}, (1, 3, 6)), ({"max_depth": 4}, (1, 2)),
                                         ({"max_leaf_nodes": 12}, (1, 2)), ({"ccp_alpha": 0.05}, (1, 2))])
def test_rf_absolute_error_matches_sklearn(extra, seeds):
    """criterion='absolute_error': weighted-median leaves and exact abs-deviation splits
    (forest_cpu.cpp Fenwick sweep); sklearn's tree on exactly binned columns, also
    through best-first (max_leaf_nodes) and ccp_alpha pruning, which read the MAE
    impurity.  Full-depth trees on other seeds hit equal-gain ties between features."""
    from sklearn.ensemble import RandomForestRegressor

    from cs230_distributed_machine_learning_amd.engine.service import refit_model

    rng = np.random.default_rng(3)
    X = rng.integers(0, 8, size=(400, 4)).astype(np.float32)
    y = np.round((1.5 * X[:, 0] - X[:, 1] + rng.standard_t(2, 400)) * 8) / 8
    for seed in seeds:
        params = {"n_estimators": 1, "bootstrap": False, "max_features": None, "criterion": "absolute_error",
                  "min_samples_leaf": 3, "random_state": seed, **extra}
        m = refit_model({"model_type": "RandomForestRegressor", "scoring": None}, params, DeviceData(X, y, False))
        sk = RandomForestRegressor(**params).fit(X, y).estimators_[0].tree_
        nodes, vals = np.asarray(m["nodes"]), np.asarray(m["vals"])
        leaves = nodes[:, 0] < 0
        ours = np.sort(vals[leaves, 1] / vals[leaves, 0])
        ref = np.sort(sk.value[sk.children_left == -1][:, 0, 0])
        assert len(ours) == len(ref)
        np.testing.assert_allclose(ours, ref, rtol=1e-9)
    fam = family_of("RandomForestRegressor")
    rp = fam.resolve("RandomForestRegressor", params, 400, 4, 1)
    assert rp["warnings"] == []


@pytest.mark.parametrize("model,kw", [
    ("RandomForestClassifier", {}),
    ("RandomForestClassifier", {"class_weight": {"0": 1.0, "1": 3.0}}),
    ("RandomForestRegressor", {}),
])
def test_rf_min_weight_fraction_leaf_matches_sklearn(model, kw):
    """min_weight_fraction_leaf: no side lighter than frac x total weight (class weights
    included), nodes lighter than twice that are leaves -- sklearn's tree on exact bins."""
    from sklearn import ensemble

    from cs230_distributed_machine_learning_amd.engine.service import refit_model

    rng = np.random.default_rng(7)
    X = rng.integers(0, 6, size=(400, 3)).astype(np.float32)
    reg = model.endswith("Regressor")
    y = (X[:, 0] * 1.5 + X[:, 1] + rng.normal(size=400)) if reg else \
        ((X[:, 0] + X[:, 1] + rng.integers(0, 3, 400)) > 6).astype(np.int64)
    skw = dict(kw)
    if "class_weight" in skw:
        skw["class_weight"] = {int(k): v for k, v in skw["class_weight"].items()}
    for frac in (0.0, 0.03, 0.12):
        params = {"n_estimators": 1, "bootstrap": False, "max_features": None, "random_state": 1,
                  "min_weight_fraction_leaf": frac}
        m = refit_model({"model_type": model, "scoring": None}, dict(params, **kw), DeviceData(X, y, not reg))
        t = getattr(ensemble, model)(**params, **skw).fit(X, y).estimators_[0].tree_
        nodes, vals = np.asarray(m["nodes"]), np.asarray(m["vals"])
        lv = nodes[:, 0] < 0
        assert lv.sum() == t.n_leaves, (frac, lv.sum(), t.n_leaves)
        if reg:
            ours = np.sort(vals[lv, 1] / vals[lv, 0])
            ref = np.sort(t.value[t.children_left == -1][:, 0, 0])
        else:
            ours = np.sort(vals[lv].sum(1))
            ref = np.sort(t.weighted_n_node_samples[t.children_left == -1])
        np.testing.assert_allclose(ours, ref, rtol=1e-4 if reg else 1e-9)   # targets are float32 here


@pytest.mark.parametrize("model,loss", [("GradientBoostingRegressor", "squared_error"),
                                        ("GradientBoostingClassifier", "log_loss")])
def test_gbrt_early_stopping_matches_sklearn(model, loss):
    """n_iter_no_change: sklearn's validation split (stratified for classifiers), its loss,
    its stopping rule -- the same number of stages and the same raw scores."""
    from sklearn import ensemble
    from sklearn.datasets import make_classification, make_regression

    from cs230_distributed_machine_learning_amd.models.boosting import gbrt_raw_numpy

    reg = model.endswith("Regressor")
    if reg:
        X, y = make_regression(400, 4, noise=25, random_state=4)
        y = np.round(y, 2)
    else:
        X, y = make_classification(400, 5, n_informative=3, n_redundant=0, flip_y=0.2, random_state=4)
    X = np.round(X, 1)
    params = {"n_estimators": 300, "loss": loss, "max_depth": 3, "learning_rate": 0.3, "n_iter_no_change": 4,
              "validation_fraction": 0.2, "random_state": 11}
    sk = getattr(ensemble, model)(**params).fit(X, y)
    assert sk.n_estimators_ < 300
    ref = sk.predict(X) if reg else sk.decision_function(X)
    dd = DeviceData(X, y, not reg, "cpu")
    dd.set_splits(np.ones((1, len(y)), np.uint8), ["full"])
    fam = family_of(model)
    rp = fam.resolve(model, params, len(y), X.shape[1], 1 if reg else 2)
    out = fam.run(dd, [FitTask(0, 0, 0, model, rp)], keep_models=True)[0]
    assert len(out.model["roots"]) == sk.n_estimators_
    got = gbrt_raw_numpy(out.model, X)[:, 0]
    # equal-gain ties between features go by the visiting order (sklearn's RNG vs ours),
    # so a deep stage can pick another of the tied splits for a few rows
    close = np.isclose(got, ref, rtol=1e-4, atol=1e-3)
    assert close.mean() >= 0.97, close.mean()


@pytest.mark.parametrize("fit_intercept", [True, False])
def test_linear_regression_positive_matches_sklearn(fit_intercept):
    """positive=True: non-negative least squares from the normal equations (NNLS on a
    Gram factor) = sklearn's nnls on the rows."""
    from sklearn.linear_model import LinearRegression

    from cs230_distributed_machine_learning_amd.engine.service import refit_model

    rng = np.random.default_rng(3)
    X = rng.normal(size=(300, 6))
    y = X @ np.array([1.5, -2.0, 0.7, 0.0, -0.3, 2.2]) + 0.5 + 0.1 * rng.normal(size=300)
    params = {"positive": True, "fit_intercept": fit_intercept}
    m = refit_model({"model_type": "LinearRegression", "scoring": None}, params, DeviceData(X, y, False))
    sk = LinearRegression(**params).fit(X, y)
    assert (m["coef"] >= 0).all()
    np.testing.assert_allclose(m["coef"], sk.coef_, atol=2e-5)
    assert abs(m["intercept"] - sk.intercept_) < 2e-5


def test_svc_break_ties_matches_sklearn():
    """break_ties=True: argmax of sklearn's one-vs-rest decision function."""
    from sklearn.datasets import make_blobs
    from sklearn.svm import SVC

    from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates

    X, y = make_blobs(240, 3, centers=4, cluster_std=3.0, random_state=2)
    grid = [{"C": 0.5, "break_ties": True}, {"C": 0.5, "break_ties": False}]
    spec = JobSpec("SVC", grid, cv=3, holdout=False, keep_models="none")
    res = run_candidates(DeviceData(X, y, True, "cpu"), spec, range(2))
    assert all(r.ok for r in res), [r.error for r in res]
    from sklearn.model_selection import StratifiedKFold, cross_val_score

    for r, g in zip(res, grid):
        ref = cross_val_score(SVC(**g), X, y, cv=StratifiedKFold(3))
        assert np.allclose(r.result["cv_scores"], ref, atol=1e-12), (g, r.result["cv_scores"], ref)


def test_knn_cosine_matches_sklearn():
    from sklearn.model_selection import StratifiedKFold, cross_val_score
    from sklearn.neighbors import KNeighborsClassifier

    from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates

    rng = np.random.default_rng(8)
    X = rng.normal(size=(300, 6))
    X[:5] = 0.0                                      # zero rows: cosine distance 1 to everything
    y = (X[:, 0] * X[:, 1] > 0).astype(np.int64)
    grid = [{"n_neighbors": k, "metric": "cosine", "weights": w} for k, w in ((5, "uniform"), (7, "distance"))]
    res = run_candidates(DeviceData(X, y, True, "cpu"), JobSpec("KNeighborsClassifier", grid, cv=3, holdout=False,
                                                                keep_models="none"), range(2))
    assert all(r.ok for r in res), [r.error for r in res]
    for r, g in zip(res, grid):
        ref = cross_val_score(KNeighborsClassifier(**g), X.astype(np.float32), y, cv=StratifiedKFold(3))
        assert np.allclose(r.result["cv_scores"], ref, atol=1e-12), (g, r.result["cv_scores"], ref)


@pytest.mark.parametrize("scoring", ["roc_auc", "neg_log_loss", "neg_brier_score", "average_precision"])
def test_rf_probability_scorers_match_sklearn(scoring):
    """Probability scorers on forests: the fits return sklearn's predict_proba (mean of the
    trees' leaf class fractions) when the job's scorer needs it."""
    from sklearn.ensemble import RandomForestClassifier
    from sklearn.model_selection import StratifiedKFold, cross_val_score

    from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates

    rng = np.random.default_rng(1)
    X = rng.integers(0, 6, size=(400, 3)).astype(np.float32)
    y = ((X[:, 0] + X[:, 1] + rng.integers(0, 4, 400)) > 7).astype(np.int64)
    # random_state 4: no equal-gain split ties between features on this table (their order is
    # sklearn's RNG vs our keyed order)
    g = {"n_estimators": 1, "bootstrap": False, "max_features": None, "min_samples_leaf": 8, "random_state": 4}
    spec = JobSpec("RandomForestClassifier", [g], cv=3, holdout=False, keep_models="none", scoring=scoring)
    res = run_candidates(DeviceData(X, y, True, "cpu"), spec, [0])
    assert res[0].ok, res[0].error
    ref = cross_val_score(RandomForestClassifier(**g), X, y, cv=StratifiedKFold(3), scoring=scoring)
    assert np.allclose(res[0].result["cv_scores"], ref, atol=1e-6), (res[0].result["cv_scores"], ref)


@pytest.mark.parametrize("scoring", ["roc_auc", "average_precision"])
def test_svc_threshold_scorers_use_decision_function(scoring):
    """sklearn's roc_auc / average_precision read SVC's decision_function (no predict_proba)."""
    from sklearn.model_selection import StratifiedKFold, cross_val_score
    from sklearn.svm import SVC

    from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates

    rng = np.random.default_rng(4)
    X = rng.normal(size=(240, 4))
    y = (X[:, 0] + 0.8 * rng.normal(size=240) > 0).astype(np.int64)
    g = {"C": 0.7, "gamma": 0.3}
    res = run_candidates(DeviceData(X, y, True, "cpu"), JobSpec("SVC", [g], cv=3, holdout=False, keep_models="none",
                                                                scoring=scoring), [0])
    assert res[0].ok, res[0].error
    ref = cross_val_score(SVC(**g), X.astype(np.float32), y, cv=StratifiedKFold(3), scoring=scoring)
    assert np.allclose(res[0].result["cv_scores"], ref, atol=1e-9), (res[0].result["cv_scores"], ref)


def test_rf_mixed_criteria_batches_keep_task_order():
    """A grid mixing absolute_error (host builder) and squared_error candidates is
    batched apart, and every output still belongs to its own task."""
    from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates

    rng = np.random.default_rng(0)
    X = rng.integers(0, 8, size=(600, 4)).astype(np.float32)
    y = X[:, 0] - X[:, 1] + rng.standard_normal(600)
    cands = [{"n_estimators": 3, "criterion": c, "max_depth": 4, "random_state": 5}
             for c in ("absolute_error", "squared_error", "absolute_error", "poisson")]
    yp = y - y.min()
    spec = JobSpec("RandomForestRegressor", cands, cv=3, holdout=False, random_state=2)
    mixed = run_candidates(DeviceData(X, yp, False, "cpu"), spec, range(4))
    for i, c in enumerate(cands):
        alone = run_candidates(DeviceData(X, yp, False, "cpu"), JobSpec("RandomForestRegressor", [c], cv=3,
                                                                         holdout=False, random_state=2), [0])[0]
        assert mixed[i].result["cv_scores"] == alone.result["cv_scores"]
    assert mixed[0].result["cv_scores"] == mixed[2].result["cv_scores"]


@pytest.mark.parametrize("model", ["RandomForestRegressor", "RandomForestClassifier"])
@pytest.mark.parametrize("extra", [{"max_depth": 5}, {"min_samples_leaf": 10}, {}])
def test_rf_monotonic_cst_matches_sklearn(model, extra):
    """monotonic_cst (sklearn >= 1.4): constrained splits keep the children's values
    ordered and inside the node's bounds, bounds meet at sklearn's middle value, node
    values are clipped -- sklearn's trees on exactly binned columns (regression at any
    depth; binary classification to the depths tested: its full-depth trees meet
    equal-gini ties between features)."""
    from sklearn.ensemble import RandomForestClassifier, RandomForestRegressor

    from cs230_distributed_machine_learning_amd.engine.service import refit_model

    is_cls = model == "RandomForestClassifier"
    if is_cls and not extra:
        pytest.skip("full-depth classification trees: equal-gain ties")
    rng = np.random.default_rng(3)
    X = rng.integers(0, 8, size=(500, 4)).astype(np.float32)
    y = np.round((0.5 * X[:, 0] - 0.3 * X[:, 1] + np.sin(X[:, 2]) + rng.standard_normal(500)) * 8) / 8
    if is_cls:
        y = (y > np.median(y)).astype(np.int64)
    Est = RandomForestClassifier if is_cls else RandomForestRegressor
    for cst in ([1, -1, 0, 0], [1, 0, -1, 1]):
        params = {"n_estimators": 1, "bootstrap": False, "max_features": None, "monotonic_cst": cst,
                  "random_state": 1, "min_samples_leaf": 2, **extra}
        m = refit_model({"model_type": model, "scoring": None}, params, DeviceData(X, y, is_cls))
        sk = Est(**params).fit(X, y).estimators_[0].tree_
        nodes, vals = np.asarray(m["nodes"]), np.asarray(m["vals"])
        leaves = nodes[:, 0] < 0
        ours = vals[leaves, 0] / vals[leaves].sum(1) if is_cls else vals[leaves, 1] / vals[leaves, 0]
        v = sk.value[sk.children_left == -1][:, 0, :]
        ref = v[:, 0] / v.sum(1) if is_cls else v[:, 0]
        assert len(ours) == len(ref)
        np.testing.assert_allclose(np.sort(ours), np.sort(ref), rtol=1e-9, atol=1e-12)
    rp = family_of(model).resolve(model, {"monotonic_cst": [1, -1, 0, 0]}, 500, 4, 2)
    assert rp["monotonic_cst"] == [1, -1, 0, 0] and rp["warnings"] == []


def test_rf_monotonic_cst_param_errors():
    from cs230_distributed_machine_learning_amd.models.base import ParamError

    fam = family_of("RandomForestClassifier")
    with pytest.raises(ParamError, match="multiclass"):
        fam.resolve("RandomForestClassifier", {"monotonic_cst": [1, 0]}, 100, 2, 3)
    with pytest.raises(ParamError, match="features"):
        fam.resolve("RandomForestClassifier", {"monotonic_cst": [1, 0, 0]}, 100, 2, 2)
    with pytest.raises(ParamError, match="-1, 0 or 1"):
        fam.resolve("RandomForestRegressor", {"monotonic_cst": [2, 0]}, 100, 2, 1)
    rp = fam.resolve("RandomForestRegressor", {"monotonic_cst": [0, 0]}, 100, 2, 1)
    assert rp["monotonic_cst"] is None
