"""Same search through this engine and through scikit-learn (reference demo_results.py /
results1.py: "distributed vs non-distributed" wall time and best parameters).

    python examples/compare_sklearn.py [rf|lr|svc|knn|gbrt] [n_rows]
"""
import os
import sys
import time

import numpy as np
from sklearn.datasets import make_classification
from sklearn.model_selection import GridSearchCV

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cs230_distributed_machine_learning_amd.data.device import DeviceData  # noqa: E402
from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates  # noqa: E402
from cs230_distributed_machine_learning_amd.search.grid import ParameterGrid  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "rf"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 5000
X, y = make_classification(n, 20, n_informative=8, random_state=0)
if which == "rf":
    from sklearn.ensemble import RandomForestClassifier as E
    name, grid = "RandomForestClassifier", {"n_estimators": [50, 100], "max_depth": [10, None],
                                            "min_samples_leaf": [1, 4]}
elif which == "lr":
    from sklearn.linear_model import LogisticRegression as E
    name, grid = "LogisticRegression", {"C": [0.01, 0.1, 1.0, 10.0, 100], "solver": ["lbfgs", "liblinear"]}
elif which == "svc":
    from sklearn.svm import SVC as E
    name, grid = "SVC", {"C": [0.3, 1, 3], "kernel": ["rbf", "poly"]}
elif which == "knn":
    from sklearn.neighbors import KNeighborsClassifier as E
    name, grid = "KNeighborsClassifier", {"n_neighbors": [3, 7, 15, 31], "weights": ["uniform", "distance"]}
else:
    from sklearn.ensemble import GradientBoostingClassifier as E
    name, grid = "GradientBoostingClassifier", {"n_estimators": [50, 100], "max_depth": [2, 3]}

import torch  # noqa: E402

dev = "cuda:0" if torch.cuda.is_available() else "cpu"
cands = list(ParameterGrid(grid))
dd = DeviceData(X, y, True, dev)
t0 = time.time()
res = run_candidates(dd, JobSpec(name, cands, cv=5, holdout=False), range(len(cands)))
t_ours = time.time() - t0
ours = np.array([r.result["mean_cv_score"] for r in res])
t0 = time.time()
ref = GridSearchCV(E(), grid, cv=5, n_jobs=-1).fit(X, y)
t_sk = time.time() - t0
sk = ref.cv_results_["mean_test_score"]
print(f"{name} {len(cands)} candidates x 5 folds on {n}x20 ({dev})")
print(f"  engine : {t_ours:8.2f} s  best {cands[int(ours.argmax())]}  {ours.max():.4f}")
print(f"  sklearn: {t_sk:8.2f} s  best {ref.best_params_}  {sk.max():.4f}")
print(f"  max |delta mean_cv| = {np.abs(ours - sk).max():.4f}")
