"""A downloaded artefact is a usable estimator (engine/model_store.py ``Predictor``).

Reference: the worker pickles the fitted sklearn estimator (aws-prod/worker/worker.py:351-356)
and ``download_best_model`` hands it to the user (DistributedLibrary/src/distributed_ml/core.py:
201-206), who then calls ``predict`` / ``predict_proba`` / ``score``.  Here the artefact is a
no-pickle ``.npz``; for every stored kind the loaded predictor must reproduce the job's own
held-out score (J4 ``accuracy`` / ``r2_score`` / ``score``) on the job's held-out rows.
"""
import numpy as np
import pytest

from cs230_distributed_machine_learning_amd.client.core import MLTaskManager
from cs230_distributed_machine_learning_amd.data.device import DeviceData
from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates
from cs230_distributed_machine_learning_amd.engine.model_store import load_predictor, save_model

sk = pytest.importorskip("sklearn")
from sklearn.datasets import make_classification, make_regression  # noqa: E402

CASES = [
    ("RandomForestClassifier", True, {"n_estimators": 12, "max_depth": 6}),
    ("RandomForestRegressor", False, {"n_estimators": 8, "max_depth": 6}),
    ("LogisticRegression", True, {"C": 1.0}),
    ("LinearRegression", False, {}),
    ("KNeighborsClassifier", True, {"n_neighbors": 5}),
    ("KNeighborsRegressor", False, {"n_neighbors": 4, "weights": "distance"}),
    ("GradientBoostingClassifier", True, {"n_estimators": 15, "max_depth": 3}),
    ("GradientBoostingRegressor", False, {"n_estimators": 15, "max_depth": 3}),
    ("SVC", True, {"C": 1.0}),
    ("SVR", False, {"C": 10.0}),
    ("PCA", False, {"n_components": 3}),
]


def _data(clf: bool, n_classes: int = 3):
    if clf:
        X, y = make_classification(400, 8, n_informative=5, n_classes=n_classes, random_state=2)
        labels = np.array(["ant", "bee", "cat", "dog"])[:n_classes]
        return X.astype(np.float32), labels[y]           # string labels: predictions come back as labels
    X, y = make_regression(400, 8, noise=4.0, random_state=3)
    return X.astype(np.float32), y.astype(np.float32)


@pytest.mark.parametrize("model,clf,params", CASES, ids=[c[0] for c in CASES])
def test_artefact_reproduces_holdout_score(tmp_path, model, clf, params):
    X, y = _data(clf)
    dd = DeviceData(X, y, clf, "cpu")
    spec = JobSpec(model, [params], cv=3, holdout=True, test_size=0.25, random_state=7, keep_models="all")
    r = run_candidates(dd, spec, [0])[0]
    assert r.ok, r.error
    path = save_model(r.model, str(tmp_path / f"{model}.npz"))
    est = load_predictor(path)
    hold = dd.split_names.index("holdout")
    te = dd.test_rows[hold].cpu().numpy()
    Xt, yt = X[te], y[te]
    if model == "PCA":
        assert est.score(Xt) == pytest.approx(r.result["score"], rel=1e-6, abs=1e-6)
        Z = est.transform(Xt)
        assert Z.shape == (len(te), 3)
        with pytest.raises(AttributeError):
            est.predict(Xt)
        return
    pred = est.predict(Xt)
    assert len(pred) == len(te)
    if clf:
        assert est.score(Xt, yt) == pytest.approx(r.result["accuracy"], abs=1e-12)
        assert set(np.unique(pred)) <= set(np.unique(y))
        if model == "SVC":
            with pytest.raises(AttributeError):
                est.predict_proba(Xt)
        else:
            P = est.predict_proba(Xt)
            assert P.shape == (len(te), 3)
            np.testing.assert_allclose(P.sum(1), 1.0, atol=1e-5)
            # the most probable class is the predicted one (ties aside)
            top = np.sort(P, 1)
            clear = top[:, -1] - top[:, -2] > 1e-6
            np.testing.assert_array_equal(est.classes_[P.argmax(1)][clear], pred[clear])
    else:
        assert est.score(Xt, yt) == pytest.approx(r.result["r2_score"], rel=1e-5, abs=1e-5)
        with pytest.raises(AttributeError):
            est.predict_proba(Xt)


def test_binary_decision_function_signs_match_predictions(tmp_path):
    X, y = _data(True, n_classes=2)
    dd = DeviceData(X, y, True, "cpu")
    for model, params in (("LogisticRegression", {"C": 0.5}), ("GradientBoostingClassifier", {"n_estimators": 10}),
                          ("SVC", {"C": 1.0})):
        spec = JobSpec(model, [params], cv=2, holdout=True, test_size=0.25, random_state=1, keep_models="all")
        r = run_candidates(dd, spec, [0])[0]
        assert r.ok, r.error
        est = MLTaskManager.load_model(save_model(r.model, str(tmp_path / f"{model}.npz")))
        dec = est.decision_function(X)
        pred = est.predict(X)
        sure = np.abs(dec) > 1e-6
        np.testing.assert_array_equal(est.classes_[(dec > 0).astype(int)][sure], pred[sure])
