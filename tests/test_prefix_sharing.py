"""Exact ensemble-prefix sharing (models/base.py ``prefix_groups``).

Fits that differ only in ``n_estimators`` and fix ``random_state`` grow the same first trees
(forests) / stages (boosting), as sklearn's estimators do.  Only the longest fit of such a
group is grown; the shorter ones are scored from its prefix.  The results must be those of
growing every fit alone (DML_PREFIX_SHARE=0): bit for bit for forests; for boosting up to the
last bits of the per-build fixed-point target grid, which depends on a build's other fits."""
import numpy as np
import pytest
from sklearn.model_selection import ParameterGrid

from cs230_distributed_machine_learning_amd.data.device import DeviceData
from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates
from cs230_distributed_machine_learning_amd.engine.model_store import load_predictor, save_model
from cs230_distributed_machine_learning_amd.models import base
from cs230_distributed_machine_learning_amd.models.base import FitTask, prefix_groups
from cs230_distributed_machine_learning_amd.models.boosting import GradientBoostingFamily
from cs230_distributed_machine_learning_amd.models.forest import ForestFamily


def _table(clf, n=900, d=7, seed=0):
    rng = np.random.RandomState(seed)
    X = np.round(rng.randn(n, d), 2).astype(np.float32)
    z = X[:, 0] + 0.7 * X[:, 1] * X[:, 2] + 0.3 * rng.randn(n)
    y = np.digitize(z, [-0.4, 0.6]) if clf else z.astype(np.float32)
    return X, y


def _fit_all(model, clf, grid, monkeypatch, tmp_path, share, dev="cpu"):
    monkeypatch.setenv("DML_PREFIX_SHARE", "1" if share else "0")
    X, y = _table(clf)
    dd = DeviceData(X, y, clf, dev)
    # classifiers scored on probabilities: the prefix fits' predict_proba path too
    spec = JobSpec(model, grid, cv=3, holdout=True, test_size=0.2, random_state=0, keep_models="all",
                   scoring="neg_log_loss" if clf else None)
    res = run_candidates(dd, spec, range(len(grid)))
    assert all(r.ok for r in res), [r.error for r in res if not r.ok]
    scores = [r.result["cv_scores"] for r in res]
    preds = [load_predictor(save_model(r.model, str(tmp_path / f"{share}_{i}.npz"))).predict(X[:300])
             for i, r in enumerate(res)]
    return scores, preds


@pytest.mark.parametrize("model,clf,grid", [
    ("RandomForestClassifier", True, {"n_estimators": [3, 5, 8], "max_depth": [4, None], "random_state": [7]}),
    ("RandomForestRegressor", False, {"n_estimators": [2, 6], "max_features": [0.5], "random_state": [1]}),
    ("GradientBoostingClassifier", True, {"n_estimators": [4, 9], "max_depth": [2, 3], "random_state": [3],
                                          "subsample": [0.8]}),
    ("GradientBoostingRegressor", False, {"n_estimators": [3, 7, 10], "loss": ["squared_error", "huber"],
                                          "random_state": [0]}),
    # forests on the GPU also nest max_depth: one leader (most and deepest trees) per split
    ("RandomForestClassifier", True, {"n_estimators": [3, 6], "max_depth": [2, 4, None], "min_samples_split": [2, 9],
                                      "random_state": [5]}),
    ("RandomForestRegressor", False, {"n_estimators": [2, 5], "max_depth": [3, None], "random_state": [2]}),
])
@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_prefix_sharing_is_exact(model, clf, grid, dev, monkeypatch, tmp_path):
    grid = list(ParameterGrid(grid))
    grown = {"forest": 0, "gbrt": 0}
    run_batch, boost = ForestFamily._run_batch, GradientBoostingFamily._boost

    def spy_batch(self, data, Xb, batch, *a, **k):
        grown["forest"] += len(batch)
        return run_batch(self, data, Xb, batch, *a, **k)

    def spy_boost(self, data, batch, *a, **k):
        grown["gbrt"] += len(batch)
        return boost(self, data, batch, *a, **k)

    monkeypatch.setattr(ForestFamily, "_run_batch", spy_batch)
    monkeypatch.setattr(GradientBoostingFamily, "_boost", spy_boost)
    s_on, p_on = _fit_all(model, clf, grid, monkeypatch, tmp_path, True, dev)
    n_on = sum(grown.values())
    grown.update(forest=0, gbrt=0)
    s_off, p_off = _fit_all(model, clf, grid, monkeypatch, tmp_path, False, dev)
    n_off = sum(grown.values())
    # fewer fits grown: one per (fold, n_estimators-free parameter set) -- on the GPU forests also
    # share max_depth, one per (fold, parameter set free of n_estimators and max_depth)
    nest = {"n_estimators"} | ({"max_depth"} if dev != "cpu" and model.startswith("RandomForest") else set())
    groups = len({repr(sorted((k, v) for k, v in c.items() if k not in nest)) for c in grid})
    assert n_off == 4 * len(grid) and n_on == 4 * groups, (n_on, n_off)
    if model.startswith("RandomForest"):
        assert s_on == s_off
        for a, b in zip(p_on, p_off):
            assert np.array_equal(np.asarray(a), np.asarray(b))
        return
    # boosting: the stage trees of one build share a fixed-point grid for their regression
    # targets (the largest target energy of the build, forest_common.h reg_exponents_counts),
    # so a fit's leaf values can move in the last bits with its batch-mates -- with or
    # without sharing (fewer fits per build here)
    np.testing.assert_allclose(np.asarray(s_on), np.asarray(s_off), rtol=0, atol=1e-9)
    for a, b in zip(p_on, p_off):
        if clf:
            assert np.mean(np.asarray(a) == np.asarray(b)) >= 0.995
        else:
            np.testing.assert_allclose(np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64),
                                       rtol=1e-9, atol=1e-9)


def test_prefix_groups_need_a_fixed_random_state():
    mk = lambda i, n, seed, split=0, **kw: FitTask(i, i, split, "RandomForestClassifier",
                                                   dict({"n_estimators": n, "seed": seed, "max_depth": 3}, **kw))
    tasks = [mk(0, 10, None), mk(1, 20, None), mk(2, 10, 5), mk(3, 30, 5), mk(4, 20, 5), mk(5, 10, 5, split=1),
             mk(6, 10, 5, max_depth=4)]
    leaders, follow = prefix_groups(tasks)
    assert [t.task_id for t in leaders] == [0, 1, 3, 5, 6]
    assert [t.task_id for t in follow[3]] == [2, 4]
    # early-stopping fits are excluded by the caller's predicate; the switch turns it off
    leaders, follow = prefix_groups(tasks, ok=lambda t: t.task_id != 3)
    assert [t.task_id for t in follow[4]] == [2]
    import os

    os.environ["DML_PREFIX_SHARE"] = "0"
    try:
        assert prefix_groups(tasks) == (tasks, {})
    finally:
        del os.environ["DML_PREFIX_SHARE"]
    assert base.prefix_groups is prefix_groups


def test_slice_planner_keeps_prefix_groups_together():
    """The runner's slices (engine/service.py plan_slices) never split a prefix group, and a
    group is priced at its longest member (the work one device batch actually does)."""
    from types import SimpleNamespace

    from cs230_distributed_machine_learning_amd.engine.service import plan_slices, prefix_units
    from cs230_distributed_machine_learning_amd.search.grid import expand_candidates

    cands = expand_candidates("GridSearchCV", {"param_grid": {"n_estimators": [50, 100, 150, 200],
                                                              "max_depth": [4, 8, 12], "min_samples_leaf": [1, 5]}})
    plan = {"model_type": "RandomForestClassifier", "candidates": cands, "cv": 5, "holdout": False,
            "base_params": {"random_state": 3}}
    units = prefix_units(plan, list(range(len(cands))))
    # forests nest n_estimators AND max_depth: one unit per min_samples_leaf
    assert len(units) == 2 and all(len(u) == 12 for u in units)
    nest = ("n_estimators", "max_depth")
    assert all(len({repr({k: v for k, v in cands[i].items() if k not in nest}) for i in u}) == 1 for u in units)
    ctl = SimpleNamespace(scheduler=SimpleNamespace(estimate=lambda mt, c: c), config=SimpleNamespace(chunk_target_s=1e-9))
    slices = plan_slices(ctl, plan, list(range(len(cands))), 10000, 10, 2, min_slices=2)
    assert sorted(map(sorted, slices)) == sorted(map(sorted, units))
    # no fixed random_state (or another family): every candidate is its own unit
    plan["base_params"] = {}
    assert len(prefix_units(plan, list(range(len(cands))))) == len(cands)
    assert len(prefix_units(dict(plan, model_type="LogisticRegression", base_params={"random_state": 1}),
                            [0, 1, 2])) == 3
    # boosting nests n_estimators only
    gb = dict(plan, model_type="GradientBoostingClassifier", base_params={"random_state": 1})
    assert len(prefix_units(gb, list(range(len(cands))))) == 6
