"""RandomForest fidelity against scikit-learn at a realistic size.

The forest builder splits on 256 quantile bins per feature where sklearn scans exact
thresholds, and draws bootstrap weights from Poisson(1) instead of a multinomial; the
acceptance rule is |delta mean CV score| <= 0.01 per candidate and the same winning
candidate.  The C++ host builder is bit-identical to the HIP builder
(tests/test_forest_gpu.py), so this CPU test pins the GPU's CV scores too.
Reference whitelist: aws-prod/worker/worker.py:38 (RandomForestClassifier)."""
import os

import numpy as np
import pytest

from cs230_distributed_machine_learning_amd.data.device import DeviceData
from cs230_distributed_machine_learning_amd.data.registry import synthetic_arrays
from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates
from cs230_distributed_machine_learning_amd.search.grid import expand_candidates

sklearn = pytest.importorskip("sklearn")


@pytest.mark.slow
@pytest.mark.timeout(900)
def test_rf_grid_cv_scores_match_sklearn_100k_x_100():
    from sklearn.ensemble import RandomForestClassifier
    from sklearn.model_selection import GridSearchCV

    X, y = synthetic_arrays("classification", 100_000, 100, 2, 10, 0, 1.0)
    grid = {"max_depth": [10, None], "min_samples_leaf": [1, 8]}
    gs = GridSearchCV(RandomForestClassifier(n_estimators=50, random_state=0, n_jobs=min(8, os.cpu_count() or 1)),
                      grid, cv=3).fit(X, y)
    ref = {(p["max_depth"], p["min_samples_leaf"]): s
           for p, s in zip(gs.cv_results_["params"], gs.cv_results_["mean_test_score"])}
    cands = [dict(c, n_estimators=50) for c in expand_candidates("GridSearchCV", {"param_grid": grid})]
    res = run_candidates(DeviceData(X, y, True, "cpu"),
                         JobSpec("RandomForestClassifier", cands, cv=3, holdout=False, keep_models="none"),
                         range(len(cands)))
    ours = {(c["max_depth"], c["min_samples_leaf"]): r.result["mean_cv_score"] for c, r in zip(cands, res)}
    for k in ref:
        assert abs(ours[k] - ref[k]) <= 0.01, (k, ours[k], ref[k])
    assert max(ours, key=ours.get) == max(ref, key=ref.get), (ours, ref)
