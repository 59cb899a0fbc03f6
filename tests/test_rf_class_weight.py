"""RandomForest class_weight (dict / "balanced" / "balanced_subsample") against sklearn.

sklearn turns class_weight into per-sample weights multiplied with the bootstrap counts
(reference whitelist aws-prod/worker/worker.py:38; sklearn/ensemble/_forest.py).  The
builders scale their integer per-class sums by the class weight exactly where those
become doubles, so an imbalanced problem's balanced accuracy moves the same way and by
the same amount as sklearn's."""
import numpy as np
import pytest

from cs230_distributed_machine_learning_amd.data.device import DeviceData
from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates

sklearn = pytest.importorskip("sklearn")


@pytest.mark.timeout(600)
def test_rf_class_weight_matches_sklearn_balanced_accuracy():
    from sklearn.datasets import make_classification
    from sklearn.ensemble import RandomForestClassifier
    from sklearn.model_selection import GridSearchCV

    X, y = make_classification(12000, 20, n_informative=6, weights=[0.9, 0.1], flip_y=0.05, random_state=1)
    X = X.astype(np.float32)
    grid = {"class_weight": [None, "balanced", "balanced_subsample", {0: 1.0, 1: 5.0}], "min_samples_leaf": [5]}
    gs = GridSearchCV(RandomForestClassifier(n_estimators=60, random_state=0, n_jobs=4), grid, cv=3,
                      scoring="balanced_accuracy").fit(X, y)
    cands = [dict(p, n_estimators=60) for p in gs.cv_results_["params"]]
    res = run_candidates(DeviceData(X, y, True, "cpu"),
                         JobSpec("RandomForestClassifier", cands, cv=3, holdout=False, keep_models="none",
                                 scoring="balanced_accuracy"), range(len(cands)))
    ref = gs.cv_results_["mean_test_score"]
    ours = np.array([r.result["mean_cv_score"] for r in res])
    assert all(r.ok and not r.result.get("warnings") for r in res)
    assert np.all(np.abs(ours - ref) <= 0.015), (ours, ref)
    # weighting the minority class raises balanced accuracy, in both implementations
    assert ours[1:].min() > ours[0] + 0.01 and ref[1:].min() > ref[0] + 0.01


def test_class_weight_table_semantics():
    from cs230_distributed_machine_learning_amd.models.base import FitTask, family_of
    from cs230_distributed_machine_learning_amd.search.cv import make_split_roles

    y = np.array(["a"] * 30 + ["b"] * 10)
    dd = DeviceData(np.random.RandomState(0).randn(40, 3).astype(np.float32), y, True, "cpu")
    roles, names = make_split_roles(y, 0, True, holdout=False)
    dd.set_splits(roles, names)
    fam = family_of("RandomForestClassifier")
    tasks = [FitTask(i, 0, 0, "RandomForestClassifier",
                     fam.resolve("RandomForestClassifier", {"n_estimators": 2, "class_weight": cw}, 40, 3, 2))
             for i, cw in enumerate([None, "balanced", {"b": 3.0}, "balanced_subsample"])]
    specs = fam._specs(tasks)
    tab = fam.class_weight_table(dd, tasks, specs)
    assert list(specs["cw_mode"]) == [0, 0, 1, 1, 1, 1, 2, 2]
    assert np.allclose(tab[0], 1.0) and np.allclose(tab[2], [40 / (2 * 30), 40 / (2 * 10)])
    assert np.allclose(tab[4], [1.0, 3.0])
