"""The batched L-BFGS / OWL-QN of LogisticRegression stays on the device.

Each fit advances its own L-BFGS state machine with masked tensor ops (models/linear.py
``LogisticFamily._solve``); the host reads one "any fit active" flag every
``DML_LR_SYNC_EVERY`` objective evaluations.  CPU: the solver's own counter plus sklearn
parity; GPU: torch's CUDA sync-debug hook counts every synchronising call of the solve."""
import warnings

import numpy as np
import pytest
import torch

from cs230_distributed_machine_learning_amd.data.device import DeviceData
from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates
from cs230_distributed_machine_learning_amd.models import linear
from cs230_distributed_machine_learning_amd.models.base import FitTask, family_of
from cs230_distributed_machine_learning_amd.search.cv import make_split_roles

sk = pytest.importorskip("sklearn")
from sklearn.datasets import make_classification  # noqa: E402
from sklearn.linear_model import LogisticRegression  # noqa: E402
from sklearn.model_selection import GridSearchCV  # noqa: E402


def _tasks(fam, dd, grid, n_splits):
    tasks = []
    for i, params in enumerate(grid):
        for s in range(n_splits):
            rp = fam.resolve("LogisticRegression", params, dd.train_counts[s], dd.d, dd.n_classes)
            tasks.append(FitTask(task_id=len(tasks), candidate=i, split=s, model_type="LogisticRegression", params=rp))
    return tasks


@pytest.mark.parametrize("n_classes", [2, 3])
def test_device_lbfgs_matches_sklearn_and_syncs_rarely(n_classes):
    X, y = make_classification(12000, 24, n_informative=8, n_classes=n_classes, random_state=2)
    X = X.astype(np.float32)
    grid = [{"C": c, "solver": s} for c in (0.01, 1.0, 100.0) for s in ("lbfgs", "liblinear")]
    dd = DeviceData(X, y, True, "cpu")
    res = run_candidates(dd, JobSpec("LogisticRegression", grid, cv=3, holdout=False), range(len(grid)))
    ours = np.array([r.result["mean_cv_score"] for r in res])
    ref = GridSearchCV(LogisticRegression(max_iter=100), {"C": [0.01, 1.0, 100.0], "solver": ["lbfgs", "liblinear"]},
                       cv=3).fit(X, y).cv_results_["mean_test_score"]
    assert np.abs(ours - ref).max() < 0.01, (ours, ref)   # same (C, solver) order as sklearn's ParameterGrid
    st = family_of("LogisticRegression").last_solve_stats
    assert st["steps"] >= st["iterations_max"] >= 5
    assert st["host_syncs"] <= st["iterations_max"], st            # <= 1 host sync per L-BFGS iteration
    assert st["host_syncs"] <= 1 + -(-st["steps"] // st["sync_every"]), st


def test_async_fits_equal_solo_fits():
    """A fit's iterates do not depend on which other fits share its batch."""
    X, y = make_classification(9000, 30, n_informative=10, random_state=4)
    dd = DeviceData(X.astype(np.float32), y, True, "cpu")
    roles, names = make_split_roles(y, 3, True, holdout=False)
    dd.set_splits(roles, names)
    fam = linear.LogisticFamily()
    grid = [{"C": 0.003}, {"C": 1.0}, {"C": 30.0, "penalty": "l1", "solver": "liblinear"}]
    both = fam.run(dd, _tasks(fam, dd, grid, 3))
    for i in range(3):
        solo = fam.run(dd, _tasks(fam, dd, [grid[i]], 3))
        for s in range(3):
            a, b = both[3 * i + s], solo[s]
            assert a.info["n_iter"] == b.info["n_iter"]
            assert torch.equal(a.pred, b.pred)


@pytest.mark.gpu
def test_device_lbfgs_sync_count_hook_gpu():
    dev = torch.device("cuda:0")
    X, y = make_classification(200000, 64, n_informative=12, random_state=5)
    dd = DeviceData(X.astype(np.float32), y, True, dev)
    roles, names = make_split_roles(y, 5, True, holdout=False)
    dd.set_splits(roles, names)
    fam = linear.LogisticFamily()
    grid = [{"C": c} for c in np.logspace(-3, 2, 8)]
    tasks = _tasks(fam, dd, grid, 5)
    b = linear._Batch(dd, tasks)
    b.mf = linear.MfmaPlan(dd, b)
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("warn")
    try:
        with warnings.catch_warnings(record=True) as rec:
            warnings.simplefilter("always")
            W, iters, n_evals = fam._solve(dd, b)
    finally:
        torch.cuda.set_sync_debug_mode(0)
    syncs = sum("synchroniz" in str(w.message) for w in rec)
    it = int(iters.max())
    assert it >= 10
    assert syncs <= it, (syncs, it, fam.last_solve_stats)     # every synchronising call, counted by torch
    assert syncs <= fam.last_solve_stats["host_syncs"] + 1


@pytest.mark.parametrize("n_classes", [2, 3])
def test_objective_at_zero_shares_group_residuals(n_classes):
    """At W = 0 every logit is 0, so fits of one (split, link, scale, class weights) group
    share their residual columns: the grouped start equals the full objective."""
    X, y = make_classification(600, 12, n_informative=6, n_classes=n_classes, random_state=4)
    dd = DeviceData(X.astype(np.float32), y, True, "cpu")
    roles, names = make_split_roles(y, 5, True, holdout=False)
    dd.set_splits(roles, names)
    fam = linear.LogisticFamily()
    grid = [{"C": c, "solver": s} for c in (0.01, 0.1, 0.3, 1.0, 3.0, 10.0) for s in ("lbfgs", "liblinear")]
    grid += [{"C": 1.0, "class_weight": "balanced"}, {"C": 2.0, "fit_intercept": False}]
    tasks = []
    for i, p in enumerate(grid):
        for sp in range(len(names)):
            rp = fam.resolve("LogisticRegression", p, dd.n, dd.d, dd.n_classes)
            tasks.append(FitTask(task_id=len(tasks), candidate=i, split=sp, model_type="LogisticRegression", params=rp))
    b = linear._Batch(dd, tasks)
    W = torch.zeros((dd.d + 1, b.M))
    f_ref, G_ref = fam._objective(dd, b, W)
    start = fam._objective_at_zero(dd, b)
    assert start is not None
    f0, G0 = start
    torch.testing.assert_close(f0, f_ref, rtol=1e-6, atol=1e-9)
    torch.testing.assert_close(G0, G_ref, rtol=1e-5, atol=1e-7)
